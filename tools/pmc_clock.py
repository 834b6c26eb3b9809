#!/usr/bin/env python3
"""Per-kernel effective shader clock and MFMA-pipe busy fraction from one rocprofv3 run that
collected counters AND a kernel trace (`rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES
--kernel-trace --output-format csv -d DIR -- cmd`).

  effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration      (MI355X_MICROARCH.md, DVFS note)
  MFMA busy       = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)
  f32 MFMA TF/s at that clock = 256 CUs * 4 SIMDs * 64 FLOP * clock

usage: tools/pmc_clock.py DIR [--flops NAME_SUBSTRING=FLOP ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 4, 8


def main():
    d = sys.argv[1]
    flops = {}
    for a in sys.argv[2:]:
        if "=" in a:
            k, v = a.split("=", 1)
            flops[k] = float(v)
    dur = {}
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f.rsplit("/", 1)[0], r["Dispatch_Id"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            names[key] = r["Kernel_Name"]
    ctr = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f.rsplit("/", 1)[0], r["Dispatch_Id"])
            ctr[key][r["Counter_Name"]] = ctr[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names.setdefault(key, r["Kernel_Name"])
    rows = defaultdict(list)
    for key, c in ctr.items():
        if key not in dur or "GRBM_GUI_ACTIVE" not in c:
            continue
        t = dur[key]
        gui = c["GRBM_GUI_ACTIVE"] / XCDS
        clk = gui / t if t > 0 else float("nan")
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * CUS * SIMDS) if gui else float("nan")
        rows[names[key]].append((t, clk, busy))
    print("| kernel | dispatches | median us | effective clock GHz | MFMA busy % | f32 peak at that clock TF/s | TF/s |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for n, v in sorted(rows.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        v.sort()
        t, clk, busy = v[len(v) // 2]
        fl = next((x for k, x in flops.items() if k in n), None)
        tf = f"{fl / t / 1e12:.1f}" if fl else ""
        short = n if len(n) < 80 else n[:77] + "..."
        print(f"| `{short}` | {len(v)} | {t * 1e6:.1f} | {clk / 1e9:.3f} | {busy * 100:.1f} | "
              f"{CUS * SIMDS * 64 * clk / 1e12:.1f} | {tf} |")


if __name__ == "__main__":
    main()
