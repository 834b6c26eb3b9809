#!/usr/bin/env python3
"""Cost probes of the Conv2 fused Winograd GEMM (winograd.hip, LDS-DMA kernel): the full Blocks 1-2
forward timed with parts of that kernel switched off through anx_wino_prio bits (4-7: no fold, no
DMA refills, no per-slice barrier, no epilogue stores; bit 0 = s_setprio, the default; bit 8 = the
interleaved-fold kernel variant). Probed
results are wrong by design; only the time differences matter. Interleaved rounds in one process."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402,F401
from anx import _native as nat  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=300)
    ap.add_argument("--bits", default="1,17,33,97,129,241")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--knob", default="anx_wino_prio", choices=["anx_wino_prio", "anx_conv1_wino_probe", "anx_set_fuse_pool1"],
                    help="which kernel's flag word the arms set (conv1: bit4 setprio, bit6 interleaved fold)")
    a = ap.parse_args()
    default = {"anx_wino_prio": 257, "anx_conv1_wino_probe": 16, "anx_set_fuse_pool1": 0}[a.knob]
    dev = torch.device("cuda", 0)
    m = AlexNetBlocks(init="rand", device=dev, max_batch=a.batch)
    x = torch.rand(a.batch, 227, 227, 3, device=dev) * 0.1
    y = torch.empty(a.batch, 13, 13, 256, device=dev)
    arms = [int(b) for b in a.bits.split(",")]
    times = {b: [] for b in arms}
    ref, diffs = None, {}
    for b in arms:
        nat.call(a.knob, b)
        m(x, out=y)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        diffs[b] = (y - ref).abs().max().item()
    for _ in range(a.rounds):
        for b in arms:
            nat.call(a.knob, b)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                m(x, out=y)
            e1.record()
            e1.synchronize()
            times[b].append(e0.elapsed_time(e1) / a.iters)
    nat.call(a.knob, default)
    base = sorted(times[arms[0]])[len(times[arms[0]]) // 2]
    for b in arms:
        t = sorted(times[b])
        ms = t[len(t) // 2]
        print(json.dumps({"bits": b, "batch": a.batch, "ms_median": round(ms, 4), "delta_us_vs_first": round((ms - base) * 1e3, 1),
                          "max_abs_diff_vs_first": diffs[b]}),
              flush=True)


if __name__ == "__main__":
    main()
