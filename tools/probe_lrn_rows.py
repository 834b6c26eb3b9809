#!/usr/bin/env python3
"""A/B of the pool2 + LRN kernels (ANX_LRN_ROWS: one wave per half output row vs 2-pixel waves):
bitwise check and device-timed forwards, alternating arms, one lane at 128 images."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402

dev = torch.device("cuda", 0)
m = AlexNetBlocks(init="rand", seed=3, device=dev, max_batch=128)
x = torch.rand((128, 227, 227, 3), device=dev) * 0.1
os.environ.pop("ANX_LRN_ROWS", None)
y0 = m(x).clone()
os.environ["ANX_LRN_ROWS"] = "1"
y1 = m(x).clone()
print(json.dumps({"bitwise_equal": bool(torch.equal(y0, y1))}), flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rnd in range(5):
    for arm in ("pairs", "rows"):
        if arm == "rows":
            os.environ["ANX_LRN_ROWS"] = "1"
        else:
            os.environ.pop("ANX_LRN_ROWS", None)
        for _ in range(5):
            m(x)
        e0.record()
        for _ in range(50):
            m(x)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"round": rnd, "arm": arm, "ms_per_forward": round(e0.elapsed_time(e1) / 50, 4)}), flush=True)
