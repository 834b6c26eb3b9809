#!/usr/bin/env python3
"""Merge rocprofv3 --pmc CSV passes into one per-kernel table (sums over dispatches) + derived rates.

usage: tools/pmc_summary.py DIR [DIR ...]   (each DIR holds a pmc_counter_collection.csv somewhere below)
"""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 4, 8  # GRBM_GUI_ACTIVE comes summed over the 8 XCDs


def main():
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((f, r["Dispatch_Id"]))
    keep = [k for k in tot if tot[k].get("GRBM_GUI_ACTIVE", 0) > 0 or tot[k].get("SQ_WAVE_CYCLES", 0) > 0]
    keep.sort(key=lambda k: -tot[k].get("GRBM_GUI_ACTIVE", 0))
    print("| kernel | dispatches | GPU cycles | MFMA busy % | VALU insts/wave-cyc | wait % | LDS bank confl % | TCC hit % | TA busy % |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in keep:
        c = tot[k]
        gui = c.get("GRBM_GUI_ACTIVE", 0) / XCDS
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * CUS * SIMDS) * 100 if gui else float("nan")
        wave = c.get("SQ_WAVE_CYCLES", 0)
        wait = c.get("SQ_WAIT_INST_ANY", 0) / wave * 100 if wave else float("nan")
        valu = c.get("SQ_INSTS_VALU", 0) / wave if wave else float("nan")
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"] * 100 if c.get("SQ_LDS_IDX_ACTIVE") else 0
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        hit = h / (h + m) * 100 if h + m else float("nan")
        ta = c.get("TA_TA_BUSY", 0) / (gui * CUS) * 100 if gui else float("nan")
        name = k if len(k) < 70 else k[:67] + "..."
        print(f"| `{name}` | {len(disp[k])} | {gui:.0f} | {mfma:.1f} | {valu:.3f} | {wait:.1f} | {lds:.1f} | {hit:.1f} | {ta:.1f} |")
    print("\nraw counters (summed over dispatches):\n")
    for k in keep:
        print(f"- `{k[:90]}`: " + ", ".join(f"{n}={v:.4g}" for n, v in sorted(tot[k].items())))


if __name__ == "__main__":
    main()
