#!/usr/bin/env python3
"""Summarise roctx marker ranges (rocprofv3 --marker-trace) of one or more rank databases into a
markdown table: per rank and range name, count / total / mean host-side ms, plus the kernel time
that fell inside each range on that rank's GPU queue.

usage: tools/marker_summary.py gpurun_out/markers/rank_*_results.db [--skip-first N]
"""
from __future__ import annotations

import argparse
import json
import sqlite3
from collections import defaultdict


def load(path: str):
    c = sqlite3.connect(path)
    regions = []
    for start, end, ext, pid in c.execute("select start, end, extdata, pid from regions"):
        try:
            name = json.loads(ext).get("message", "?")
        except (ValueError, TypeError):
            name = "?"
        regions.append((name, start, end, pid))
    kernels = [(s, e) for s, e in c.execute("select start, end from kernels")]
    return regions, kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--skip-first", type=int, default=1, help="ranges of each name to skip (cold step)")
    a = ap.parse_args()
    print("| rank (pid) | range | count | host ms total | host ms mean | kernel ms inside |")
    print("|---|---|---:|---:|---:|---:|")
    for db in a.dbs:
        regions, kernels = load(db)
        seen = defaultdict(int)
        agg = defaultdict(lambda: [0, 0.0, 0.0])
        for name, s, e, pid in sorted(regions, key=lambda r: r[1]):
            seen[name] += 1
            if seen[name] <= a.skip_first:
                continue
            k = sum(max(0, min(e, ke) - max(s, ks)) for ks, ke in kernels)
            g = agg[(pid, name)]
            g[0] += 1
            g[1] += (e - s) / 1e6
            g[2] += k / 1e6
        for (pid, name), (n, t, k) in sorted(agg.items()):
            print(f"| {pid} | {name} | {n} | {t:.3f} | {t / n:.4f} | {k:.3f} |")


if __name__ == "__main__":
    main()
