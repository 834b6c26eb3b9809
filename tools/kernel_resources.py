#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy report of a HIP source for gfx950 (compile-time; no GPU).

usage: tools/kernel_resources.py csrc/src/hip/conv_mfma.hip [--filter conv_mfma] [--src-override FILE]
Parses clang's -Rpass-analysis=kernel-resource-usage remarks.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    ap.add_argument("--include", default=os.path.join(ROOT, "csrc", "include"))
    a = ap.parse_args()
    cmd = ["/opt/rocm/llvm/bin/clang++", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{a.include}",
           "--cuda-device-only", "-c", a.src, "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    demangled = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                               capture_output=True, text=True).stdout.splitlines()
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'scratch':>7s} {'LDS':>6s} {'occ':>4s}")
    for r, d in zip(rows, demangled):
        if a.filter and a.filter not in d:
            continue
        d = re.sub(r"\(anonymous namespace\)::|anx::hip::", "", d)
        print(f"{d[:70]:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>5s} "
              f"{r.get('ScratchSize', '?'):>7s} {r.get('LDS Size', '?'):>6s} {r.get('Occupancy', '?'):>4s}")


if __name__ == "__main__":
    sys.exit(main())
