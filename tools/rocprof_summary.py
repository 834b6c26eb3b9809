#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (``-d DIR -o NAME`` writes NAME_results.db, or a
``--output-format csv`` kernel_trace.csv) into a per-kernel markdown table.

usage: tools/rocprof_summary.py <results.db|kernel_trace.csv> [--steps N] [--flops-per-step F]
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3
from collections import defaultdict


def load(path):
    import os
    if os.path.isdir(path):  # a rocprofv3 -d DIR: its kernel_trace csv or results db
        import glob
        hits = glob.glob(os.path.join(path, "*kernel_trace.csv")) or glob.glob(os.path.join(path, "*.db"))
        if not hits:
            raise SystemExit(f"no kernel trace under {path}")
        path = hits[0]
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e, vg, agv, lds, gx, wx in c.execute(
                "select name, start, end, vgpr_count, accum_vgpr_count, lds_size, grid_x, workgroup_x from kernels"):
            rows.append((name, (e - s) / 1e3, vg, agv, lds, gx // max(wx, 1)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                rows.append((r["Kernel_Name"], d, r.get("VGPR_Count", ""), r.get("Accum_VGPR_Count", ""),
                             r.get("LDS_Block_Size", ""), ""))
    return rows


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", name)  # drop the argument list
    return name.replace("anx::hip::", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="timed+warmup steps in the trace (per-step column)")
    args = ap.parse_args()
    agg = defaultdict(lambda: [0, 0.0, None])
    for name, us, vg, agv, lds, wgs in load(args.path):
        a = agg[short(name)]
        a[0] += 1
        a[1] += us
        a[2] = (vg, agv, lds, wgs)
    tot = sum(a[1] for a in agg.values())
    print("| kernel | calls | avg us | total ms | share | vgpr/agpr | lds B | workgroups |")
    print("|---|---:|---:|---:|---:|---|---:|---:|")
    for k, (n, us, meta) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        vg, agv, lds, wgs = meta
        print(f"| `{k}` | {n} | {us / n:.1f} | {us / 1e3:.3f} | {100 * us / tot:.1f}% | {vg}/{agv} | {lds} | {wgs} |")
    print(f"\ntotal kernel time {tot / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
