#!/usr/bin/env python3
"""Probe: AlexNetBlocks.forward_async over K forwards (fresh start each repetition): ms per forward and
the per-lane finish times of every forward (device events), to see the lanes' phase and drift."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402,F401
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
m = AlexNetBlocks(init="rand", seed=1, device=dev, max_batch=B, lanes=2)
x = torch.rand(B, 227, 227, 3, device=dev) * 0.1
y = m(x)
big = AlexNetBlocks(m.weights, device=dev, max_batch=600, lanes=2) if len(sys.argv) > 2 else None
xb = torch.rand(600, 227, 227, 3, device=dev) * 0.1 if big else None
yb = big(xb) if big else None
for K in (10, 30, 30, 100, 30):
    torch.cuda.synchronize()
    if big is not None:  # a large different-model run right before (the sweep's slow case)
        for _ in range(10):
            big.forward_async(xb, yb)
        big.join()
        torch.cuda.synchronize()
    ev = {0: [], 1: []}

    def on_lane(i, lo, hi):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev[i].append(e)

    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        m.forward_async(x, y, on_lane=on_lane)
    m.join()
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    e1.synchronize()
    t = {i: [round(e0.elapsed_time(e), 3) for e in ev[i]] for i in ev}
    print(json.dumps({"B": B, "K": K, "ms_per_forward": round(e0.elapsed_time(e1) / K, 4),
                      "lane0_end_ms": t[0][:8] + t[0][-3:], "lane1_end_ms": t[1][:8] + t[1][-3:]}), flush=True)
