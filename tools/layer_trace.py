"""Per-dispatch kernel times of the last bench step from a rocprofv3 kernel-trace database, in launch
order (one line per layer kernel): which layer of a step costs what.

Usage: python tools/layer_trace.py gpurun_out/full_prof/run_results.db [--last N]
"""
import argparse
import re
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=13, help="dispatches in one step")
    ap.add_argument("--steps", type=int, default=5, help="average over this many trailing steps")
    ap.add_argument("--first", default="conv1", help="regex naming a step's first kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels order by start"))
    n = a.last
    starts = [i for i, r in enumerate(rows) if re.search(a.first, r[0]) and i + n <= len(rows)]
    starts = starts[-a.steps:]
    tail = [r for st in starts for r in rows[st:st + n]]
    a.steps = len(starts)
    print(f"| # | kernel | avg us (last {a.steps} steps) | workgroups |")
    print("|---:|---|---:|---:|")
    tot = 0.0
    for i in range(n):
        name, _, gx, gy, gz, wx = tail[i]
        us = sum(tail[i + s * n][1] for s in range(a.steps)) / a.steps / 1000
        tot += us
        short = re.sub(r"anx::hip::|\(anonymous namespace\)::|^void ", "", name)
        short = re.sub(r"\(.*$", "", short)[:70]
        print(f"| {i} | `{short}` | {us:.1f} | {gx // wx * gy * gz} |")
    print(f"\nsum {tot:.1f} us per step")


if __name__ == "__main__":
    main()
