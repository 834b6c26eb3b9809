#!/usr/bin/env python3
"""Forward latency / throughput of the Blocks 1-2 engine over batch sizes (one process, one GPU,
interleaved rounds as the CDNA guide's methodology rule 24 asks)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,16,32,64,128,256")
    ap.add_argument("--impl", default="mfma")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bs = [int(b) for b in a.batches.split(",")]
    m = AlexNetBlocks(init="rand", device=dev, impl=a.impl, max_batch=max(bs))
    xs = {b: torch.rand(b, 227, 227, 3, device=dev) * 0.1 for b in bs}
    ys = {b: torch.empty(b, 13, 13, 256, device=dev) for b in bs}
    res = {b: [] for b in bs}
    for b in bs:
        m(xs[b], out=ys[b])
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for b in bs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                m(xs[b], out=ys[b])
            e1.record()
            e1.synchronize()
            res[b].append(e0.elapsed_time(e1) / a.iters)
    f = anx.flops_per_image()
    for b in bs:
        ms = sorted(res[b])[len(res[b]) // 2]
        print(json.dumps({"batch": b, "impl": a.impl, "ms_median": round(ms, 4), "ms_min": round(min(res[b]), 4),
                          "img_per_s": round(b / ms * 1e3, 1), "tflops": round(b * f / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
