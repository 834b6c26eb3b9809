#!/usr/bin/env python3
"""Per-kernel effective shader clock and MFMA-pipe busy fraction from one rocprofv3 run that
collected counters AND a kernel trace (`rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES
--kernel-trace --output-format csv -d DIR -- cmd`).

  effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration      (MI355X_MICROARCH.md, DVFS note)
  MFMA busy       = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)
  f32 MFMA TF/s at that clock = 256 CUs * 4 SIMDs * 64 FLOP * clock

  FETCH_SIZE / WRITE_SIZE (KB, when collected): HBM-side bytes per dispatch and the GB/s they imply

usage: tools/pmc_clock.py DIR [DIR2 ...] [NAME_SUBSTRING=FLOP ...]   (dirs are merged by kernel name)
"""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 4, 8


def main():
    dirs = [a for a in sys.argv[1:] if "=" not in a]
    flops = {}
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=", 1)
            flops[k] = float(v)
    dur = {}
    names = {}
    files = lambda pat: [f for d in dirs for f in glob.glob(os.path.join(d, "**", pat), recursive=True)]  # noqa: E731
    for f in files("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            key = (f.rsplit("/", 1)[0], r["Dispatch_Id"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            names[key] = r["Kernel_Name"]
    ctr = defaultdict(dict)
    for f in files("*counter_collection.csv"):
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
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (gui * CUS * SIMDS) if gui else float("nan")
        rows[names[key]].append((t, clk, busy, c.get("FETCH_SIZE"), c.get("WRITE_SIZE")))
    print("| kernel | dispatches | median us | effective clock GHz | MFMA busy % | f32 peak at that clock TF/s | TF/s "
          "| fetch MB | write MB | HBM GB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    med = lambda xs: sorted(xs)[len(xs) // 2] if xs else None  # noqa: E731
    for n, v in sorted(rows.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        t = med([x[0] for x in v])
        clk = med([x[1] for x in v])
        busy = med([x[2] for x in v if x[2] == x[2]])
        fe = med([x[3] for x in v if x[3] is not None])
        wr = med([x[4] for x in v if x[4] is not None])
        fl = next((x for k, x in flops.items() if k in n), None)
        tf = f"{fl / t / 1e12:.1f}" if fl else ""
        short = n if len(n) < 80 else n[:77] + "..."
        mb = lambda kb: f"{kb / 1024:.1f}" if kb is not None else ""  # noqa: E731
        bw = sum(x for x in (fe, wr) if x is not None) * 1024 / t / 1e9 if (fe is not None or wr is not None) else None
        # FETCH and WRITE come from different passes: the GB/s pairs their medians with the pass-merged median time
        print(f"| `{short}` | {len(v)} | {t * 1e6:.1f} | {clk / 1e9:.3f} | "
              f"{'' if busy is None else f'{busy * 100:.1f}'} | {CUS * SIMDS * 64 * clk / 1e12:.1f} | {tf} | "
              f"{mb(fe)} | {mb(wr)} | {'' if bw is None else f'{bw:.0f}'} |")


if __name__ == "__main__":
    main()
