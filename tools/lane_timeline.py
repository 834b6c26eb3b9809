#!/usr/bin/env python3
"""How busy the GPU is inside the bench's steady state, from a rocprofv3 kernel trace (csv).

For the last ``--window`` dispatches of the Blocks kernels (default: the last 40 steps x 2 lanes x 4
kernels) it reports, over the window's wall span: the time at least one kernel runs (union), the time two or
more run at once, the idle gaps (no kernel running) and, per queue (one per lane stream), the sum of its
kernels' durations. A step is 2 lanes x (conv1_fused, pool_wino_in, gemm16, maxpool_lrn256); idle gaps are
host launch / join latency the lanes did not hide.

usage: python tools/lane_timeline.py gpurun_out/r06lt/prof/bench_kernel_trace.csv [--window N]
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict

PAT = re.compile(r"conv1_fused|pool_wino_in|gemm16|maxpool_lrn256")


def short(name: str) -> str:
    m = PAT.search(name)
    return m.group(0) if m else name[:40]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window", type=int, default=320, help="trailing Blocks dispatches analysed")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            if PAT.search(r["Kernel_Name"]):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                             short(r["Kernel_Name"])))
    rows.sort()
    rows = rows[-a.window:]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    span = t1 - t0
    # sweep line over start / end events
    ev = sorted([(s, 1) for s, _, _, _ in rows] + [(e, -1) for _, e, _, _ in rows])
    busy = multi = 0
    gaps = []
    depth, last = 0, t0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        if depth == 0 and t > last:
            gaps.append(t - last)
        depth += d
        last = t
    per_q = defaultdict(float)
    per_k = defaultdict(list)
    for s, e, q, k in rows:
        per_q[q] += e - s
        per_k[k].append(e - s)
    us = lambda ns: ns / 1000.0
    print(f"window: {len(rows)} dispatches, {us(span):.1f} us wall")
    print(f"any kernel running: {us(busy):.1f} us ({100 * busy / span:.1f} %); two or more: {us(multi):.1f} us "
          f"({100 * multi / span:.1f} %)")
    gaps.sort()
    print(f"idle gaps: {len(gaps)}, total {us(sum(gaps)):.1f} us, largest {us(gaps[-1]) if gaps else 0:.1f} us, "
          f"median {us(gaps[len(gaps) // 2]) if gaps else 0:.2f} us")
    for q, v in sorted(per_q.items()):
        print(f"queue {q}: kernels {us(v):.1f} us ({100 * v / span:.1f} % of the window)")
    print("| kernel | dispatches | median us | sum us |")
    print("|---|---:|---:|---:|")
    for k, v in sorted(per_k.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"| `{k}` | {len(v)} | {us(v[len(v) // 2]):.1f} | {us(sum(v)):.1f} |")


if __name__ == "__main__":
    main()
