#!/usr/bin/env python3
"""Probe: per-step lane join cost. Times K steps of the 2-lane 128-image Blocks forward three ways:
joined (AlexNetBlocks.forward: fork/join on the current stream every step, the bench's step),
free-running lanes (each lane's engine enqueued on its own stream, one join at the end), and
free-running with lane 1 started half a step late. Event-timed on the device, same buffers."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import anx  # noqa: E402,F401
from anx.models.alexnet_blocks import AlexNetBlocks, full_plan  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
K = 200
m = AlexNetBlocks(init="rand", seed=1, device=dev, max_batch=B, lanes=2)
x = torch.rand(B, 227, 227, 3, device=dev) * 0.1
y = m(x)
plan = full_plan(m.H, m.W, m.b1, m.b2)
h = B // 2
engines = [m, m._lanes[0]]
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def run(mode):
    torch.cuda.synchronize()
    for _ in range(50):
        m(x, out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cur = torch.cuda.current_stream()
    if mode == "joined":
        for _ in range(K):
            m(x, out=y)
    else:
        for st in streams:
            st.wait_stream(cur)
        evs = [[torch.cuda.Event() for _ in range(2)] for _ in range(2)]  # [lane][parity]
        for k in range(K if mode == "interlock" else 0):
            for i, (eng, st) in enumerate(zip(engines, streams)):
                with torch.cuda.stream(st):
                    # stage 1 of lane i waits for the other lane's latest stage 1 (alternation)
                    if i == 1:
                        st.wait_event(evs[0][k & 1])
                    elif k > 0:
                        st.wait_event(evs[1][(k - 1) & 1])
                    eng.stage1(x[i * h:(i + 1) * h], plan)
                    evs[i][k & 1].record(st)
                    eng.stage2(h, plan, y[i * h:(i + 1) * h])
        for k in range(0 if mode == "interlock" else K):
            for i, (eng, st) in enumerate(zip(engines, streams)):
                with torch.cuda.stream(st):
                    if mode == "offset" and k == 0 and i == 0:
                        # lane 1 starts when lane 0's stage 1 (conv1 + pool1) of the first step is done
                        eng.stage1(x[:h], plan)
                        ev = torch.cuda.Event()
                        ev.record(st)
                        eng.stage2(h, plan, y[:h])
                        continue
                    if mode == "offset" and k == 0 and i == 1:
                        st.wait_event(ev)
                    eng.tile_forward(x[i * h:(i + 1) * h], plan, y[i * h:(i + 1) * h])
        for st in streams:
            cur.wait_stream(st)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / K
    return {"mode": mode, "ms_per_step": round(ms, 4), "img_per_s": round(B / ms * 1e3, 1)}


for rep in range(2):
    for mode in ("joined", "free", "offset", "interlock"):
        print(json.dumps(run(mode)), flush=True)
