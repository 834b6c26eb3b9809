#!/usr/bin/env python3
"""Forward latency / throughput of the Blocks 1-2 engine over batch sizes (one process, one GPU,
interleaved rounds as the CDNA guide's methodology rule 24 asks). --lanes L runs batches of at
least L * 64 images as L stream lanes; --async times them as the bench's step does
(AlexNetBlocks.forward_async: free-running lanes, joined once per timed round)."""
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
    ap.add_argument("--lanes", type=int, default=1)
    ap.add_argument("--async", dest="async_", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bs = [int(b) for b in a.batches.split(",")]
    from anx.models.alexnet_blocks import LANE_MIN
    base = AlexNetBlocks(init="rand", device=dev, impl=a.impl, max_batch=max(bs))
    models = {b: (AlexNetBlocks(base.weights, device=dev, impl=a.impl, max_batch=b, lanes=a.lanes)
                  if a.lanes > 1 and b >= a.lanes * LANE_MIN else base) for b in bs}
    xs = {b: torch.rand(b, 227, 227, 3, device=dev) * 0.1 for b in bs}
    ys = {b: torch.empty(b, 13, 13, 256, device=dev) for b in bs}
    res = {b: [] for b in bs}
    for b in bs:
        models[b](xs[b], out=ys[b])
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for b in bs:
            m = models[b]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                if a.async_:
                    m.forward_async(xs[b], ys[b])
                else:
                    m(xs[b], out=ys[b])
            if a.async_:
                m.join()
            e1.record()
            e1.synchronize()
            res[b].append(e0.elapsed_time(e1) / a.iters)
    f = anx.flops_per_image()
    for b in bs:
        ms = sorted(res[b])[len(res[b]) // 2]
        print(json.dumps({"batch": b, "impl": a.impl, "lanes": models[b].lane_count(), "async": a.async_,
                          "ms_median": round(ms, 4), "ms_min": round(min(res[b]), 4),
                          "img_per_s": round(b / ms * 1e3, 1), "tflops": round(b * f / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
