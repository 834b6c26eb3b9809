#!/usr/bin/env python3
"""In-process A/B of engine kernel knobs on the full Blocks 1-2 forward (CDNA guide §5.4 rule 24:
interleaved rounds in ONE process, report median and min).

Every arm is its own model (own engine, own knobs: anx/knobs.hpp), so arms never touch shared state.

usage: tools/ab_variants.py --arms "|conv1_occ=3|conv2_occ=1" --batch 128 --lanes 2
An arm is ';'-separated name=value pairs over the defaults (empty arm = defaults); '|' separates
arms. Names: anx.utils.tuning.KNOBS (algorithm knobs take auto/direct/winograd). --lanes L runs
every arm as L stream lanes; max_abs_diff_vs_arm0 says which arms are bit-identical to arm 0."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402


def parse_arm(spec: str) -> dict:
    out = {}
    for kv in filter(None, (p.strip() for p in spec.split(";"))):
        k, v = kv.split("=", 1)
        out[k.strip()] = v.strip() if k.strip().endswith("_algo") and not v.strip().lstrip("-").isdigit() else int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="|conv1_occ=3")
    ap.add_argument("--batch", type=int, default=300)
    ap.add_argument("--lanes", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    arms = [parse_arm(s) for s in a.arms.split("|")]
    x = torch.rand(a.batch, 227, 227, 3, device=dev) * 0.1
    models, ref = [], None
    for knobs in arms:
        kn = dict(knobs)
        prio = kn.pop("lane_prio", 0)  # not a kernel knob: stream priority of the side lanes
        m = AlexNetBlocks(init="rand", device=dev, max_batch=a.batch, lanes=a.lanes, knobs=kn, lane_priority=prio)
        y = m(x)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        models.append((m, torch.empty_like(y), (y - ref).abs().max().item()))
    times = [[] for _ in arms]
    for _ in range(a.rounds):
        for i, (m, y, _) in enumerate(models):
            m(x, out=y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                m(x, out=y)
            e1.record()
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.iters)
    f = anx.flops_per_image()
    for knobs, t, (_, _, err) in zip(arms, times, models):
        med = sorted(t)[len(t) // 2]
        print(json.dumps({"arm": knobs, "batch": a.batch, "lanes": a.lanes, "ms_median": round(med, 4),
                          "ms_min": round(min(t), 4), "img_per_s": round(a.batch / med * 1e3, 1),
                          "direct_equiv_tflops": round(a.batch * f / med / 1e9, 2), "max_abs_diff_vs_arm0": err}),
              flush=True)


if __name__ == "__main__":
    main()
