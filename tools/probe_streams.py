#!/usr/bin/env python3
"""Throughput of the Blocks 1-2 engine when the batch is split over S concurrent HIP streams, one
engine (own workspace, same weights) per stream, against the single-stream launch. The memory-bound
transforms/pools of one stream can then fill the CUs the MFMA GEMMs of another leave idle in their
tail waves. Interleaved rounds, CUDA events, medians (cdna_hip_programming.md methodology)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402
from anx.parallel.plan import full_plan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1x300,2x150,2x150s,2x128,2x128s,2x192,2x192s,1x600,2x300,2x300s")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfgs = [tuple(int(v) for v in c.rstrip("s").split("x")) + (int(c.endswith("s")),) for c in a.configs.split(",")]
    smax = max(c[0] for c in cfgs)
    bmax = max(c[1] for c in cfgs)
    base = AlexNetBlocks(init="rand", seed=3, device=dev, max_batch=bmax)
    models = [base] + [AlexNetBlocks(base.weights, device=dev, max_batch=bmax) for _ in range(smax - 1)]
    streams = [torch.cuda.Stream() for _ in range(smax)]
    xs = [torch.rand(bmax, 227, 227, 3, device=dev) * 0.1 for _ in range(smax)]
    ys = [torch.empty(bmax, 13, 13, 256, device=dev) for _ in range(smax)]

    plan = full_plan(227, 227, base.b1, base.b2)

    def step(s, b, skew=0):
        cur = torch.cuda.current_stream()
        ev = None
        for i in range(s):
            streams[i].wait_stream(cur)
            with torch.cuda.stream(streams[i]):
                if not skew:
                    models[i](xs[i][:b], out=ys[i][:b])
                    continue
                # skewed: stream i starts its block 1 once stream i-1's block 1 is done, so block 1
                # (conv1 + pool1) of one half runs beside block 2 (conv2 + pool2/LRN) of the other
                if ev is not None:
                    streams[i].wait_event(ev)
                models[i].stage1(xs[i][:b], plan)
                ev = torch.cuda.Event()
                ev.record(streams[i])
                models[i].stage2(b, plan, out=ys[i][:b])
        for i in range(s):
            cur.wait_stream(streams[i])

    for c in cfgs:
        step(*c)
    torch.cuda.synchronize()
    # same images through 1 stream and S streams give the same outputs (independent engines)
    if smax >= 2:
        ref = models[0](xs[1][:8]).clone()
        for sk in (0, 1):
            ys[1].zero_()
            step(2, 8, sk)
            torch.cuda.synchronize()
            assert torch.equal(ref, ys[1][:8]), sk
    res = {c: [] for c in cfgs}
    for _ in range(a.rounds):
        for c in cfgs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                step(*c)
            e1.record()
            e1.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.iters)
    for s, b, sk in cfgs:
        ms = sorted(res[(s, b, sk)])[len(res[(s, b, sk)]) // 2]
        print(json.dumps({"streams": s, "batch_per_stream": b, "skew": sk, "images": s * b, "ms_median": round(ms, 4),
                          "img_per_s": round(s * b / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
