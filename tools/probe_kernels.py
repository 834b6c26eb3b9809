#!/usr/bin/env python3
"""Cost probes of the conv1 Winograd GEMM: time the conv1 kernels alone (anx_conv1_wino on resident
buffers) with parts of the kernel switched off (fold, DMA refills). Results of probed runs are
wrong by design; only the timings matter. Interleaved rounds in one process (guide rule 24)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402,F401
from anx import _native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=300)
    ap.add_argument("--probes", default="0,1,2,3")
    ap.add_argument("--cfgs", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = a.batch
    x = torch.rand(N, 227, 227, 3, device=dev) * 0.1
    w = (torch.rand(96, 3, 11, 11) - 0.5) * 0.02
    b = torch.zeros(96, device=dev)
    y = torch.empty(N, 55, 55, 96, device=dev)
    arms = [(int(c), int(p)) for c in a.cfgs.split(",") for p in a.probes.split(",")]
    times = {arm: [] for arm in arms}
    s = nat.stream_ptr(dev)
    for _ in range(a.rounds):
        for cfg, probe in arms:
            nat.call("anx_conv1_wino_cfg", cfg)
            nat.call("anx_conv1_wino_probe", probe)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                nat.call("anx_conv1_wino", x.data_ptr(), N, 227, 227, w.data_ptr(), 96, 11, b.data_ptr(), y.data_ptr(),
                         1, s)
            e1.record()
            e1.synchronize()
            times[(cfg, probe)].append(e0.elapsed_time(e1) / a.iters)
    nat.call("anx_conv1_wino_probe", 16)
    nat.call("anx_conv1_wino_cfg", 4)
    for arm, t in times.items():
        t = sorted(t)
        print(json.dumps({"cfg": arm[0], "probe": arm[1], "batch": N, "ms_median": round(t[len(t) // 2], 4),
                          "note": "includes weight transform upload + V alloc per call"}))


if __name__ == "__main__":
    main()
