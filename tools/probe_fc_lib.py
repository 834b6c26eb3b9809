#!/usr/bin/env python3
"""How fast is a library GEMM (torch.nn.functional.linear -> hipBLASLt on ROCm) on the full model's FC
shapes at 256 images, bf16 in / fp32 accumulate, against our wide-tile split-K FC kernels
(FC6 36 us, FC7 20 us, FC8 12 us + two ~5 us reduces: profiles/r04_full_bf16_layers_pool1.md)."""
import json
import time

import torch
import torch.nn.functional as F


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda", 0)
    M = 256
    for name, K, N in (("fc6", 9216, 4096), ("fc7", 4096, 4096), ("fc8", 4096, 1000)):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.01
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        us = bench(lambda: F.relu(F.linear(x, w, b)))
        us_plain = bench(lambda: F.linear(x, w, b))
        print(json.dumps({"layer": name, "M": M, "K": K, "N": N, "us_linear_relu": round(us, 1),
                          "us_linear": round(us_plain, 1), "weight_tb_s": round(N * K * 2 / us_plain / 1e6, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
