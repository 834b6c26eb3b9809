#!/usr/bin/env python3
"""In-process A/B of the engine's per-stage launch chunking (anx_set_stage_chunks): the batch is
run as chunks of c1 images through Conv1+Pool1 and c2 images through Conv2+Pool2+LRN, reusing one
set of Winograd V buffers per chunk (Infinity-Cache residency vs wave quantization). Interleaved
rounds in one process; results are bit-identical across arms (checked).

usage: tools/ab_chunks.py --batch 300 --arms "0:0,60:100,100:100,150:150"
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402
from anx import _native as nat  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="0:0,60:100,100:100,150:150")
    ap.add_argument("--batch", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    arms = [tuple(int(v) for v in s.split(":")) for s in a.arms.split(",")]
    m = AlexNetBlocks(init="rand", device=dev, max_batch=a.batch)
    x = torch.rand(a.batch, 227, 227, 3, device=dev) * 0.1
    y = torch.empty(a.batch, 13, 13, 256, device=dev)
    ref, diffs = None, {}
    for arm in arms:
        nat.call("anx_set_stage_chunks", *arm)
        m(x, out=y)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        diffs[arm] = (y - ref).abs().max().item()
    times = {arm: [] for arm in arms}
    for _ in range(a.rounds):
        for arm in arms:
            nat.call("anx_set_stage_chunks", *arm)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                m(x, out=y)
            e1.record()
            e1.synchronize()
            times[arm].append(e0.elapsed_time(e1) / a.iters)
    nat.call("anx_set_stage_chunks", 0, 0)
    for arm in arms:
        t = sorted(times[arm])
        ms = t[len(t) // 2]
        print(json.dumps({"chunk1": arm[0], "chunk2": arm[1], "batch": a.batch, "ms_median": round(ms, 4),
                          "ms_min": round(t[0], 4), "img_per_s": round(a.batch / ms * 1e3, 1),
                          "max_abs_diff_vs_first": diffs[arm]}), flush=True)


if __name__ == "__main__":
    main()
