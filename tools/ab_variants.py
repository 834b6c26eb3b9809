#!/usr/bin/env python3
"""In-process A/B of conv tile variants on the full Blocks 1-2 forward (CDNA guide §5.4 rule 24:
interleaved rounds in ONE process, report median and min).

usage: tools/ab_variants.py --arms "0:1,5:6,7:8" --batch 128
each arm = <vec4 variant>:<scalar variant>[:<conv2 algo 0 auto|1 direct|2 winograd>[:<wino fused cfg>
[:<conv1 algo 0 auto|1 direct|2 winograd>[:<conv1 winograd ring cfg 0..2>]]]] (-1 = heuristic)."""
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
    ap.add_argument("--arms", default="-1:-1:1,-1:-1:2")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    defaults = [-1, -1, 0, 7, 0, 4]
    arms = []
    for spec in a.arms.split(","):
        f = [int(v) for v in spec.split(":")]
        arms.append(tuple(f + defaults[len(f):]))

    def force(arm):
        v4, sc, al, fc, c1, c1c = arm
        nat.call("anx_conv_force_variant", 0, v4)
        nat.call("anx_conv_force_variant", 1, sc)
        nat.call("anx_set_conv2_algo", al)
        nat.call("anx_wino_fused_cfg", fc)
        nat.call("anx_set_conv1_algo", c1)
        nat.call("anx_conv1_wino_cfg", c1c)
    models = []
    x = torch.rand(a.batch, 227, 227, 3, device=dev) * 0.1
    ref = None
    for arm in arms:
        force(arm)
        m = AlexNetBlocks(init="rand", device=dev, max_batch=a.batch)
        y = m(x)  # packs weights for the forced variants
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        err = (y - ref).abs().max().item()
        models.append((m, torch.empty_like(y), err))
    times = [[] for _ in arms]
    for _ in range(a.rounds):
        for i, (m, y, _) in enumerate(models):
            # the variant is chosen at plan time (every call): force it for this arm's launches
            force(arms[i])
            m(x, out=y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                m(x, out=y)
            e1.record()
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.iters)
    force(tuple(defaults))
    f = anx.flops_per_image()
    for arm, t, (_, _, err) in zip(arms, times, models):
        med = sorted(t)[len(t) // 2]
        print(json.dumps({"arm": ":".join(str(v) for v in arm), "batch": a.batch, "ms_median": round(med, 4), "ms_min": round(min(t), 4),
                          "img_per_s": round(a.batch / med * 1e3, 1), "tflops": round(a.batch * f / med / 1e9, 2),
                          "max_abs_diff_vs_arm0": err}))


if __name__ == "__main__":
    main()
