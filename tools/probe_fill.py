#!/usr/bin/env python3
"""How much of a short timed window is pipeline fill: the bench's dp step (2 free-running lanes,
128 images, rotated inputs) timed as repeated windows of K steps, each bracketed by a device
synchronisation (as bench.py's timed region is), for K = 5, 20, 200. The fill cost per window is
total(K) - K * T, with T from the long windows.

usage: tools/probe_fill.py [--lanes 2] [--stagger-after stage1|none]"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = AlexNetBlocks(init="rand", seed=1, device=dev, max_batch=a.batch, lanes=a.lanes)
    xs = [torch.rand((a.batch, 227, 227, 3), device=dev) * 0.1 for _ in range(4)]
    y = torch.empty((a.batch, 13, 13, 256), device=dev)
    k = 0
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:  # clock settle
        m.forward_async(xs[k % 4], y)
        k += 1
    torch.cuda.synchronize()
    for K in (5, 20, 200, 20, 5, 200):
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                m.forward_async(xs[k % 4], y)
                k += 1
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            print(json.dumps({"K": K, "ms": round(dt, 4), "ms_per_step": round(dt / K, 4)}), flush=True)


if __name__ == "__main__":
    main()
