#!/usr/bin/env python3
"""Root-ingest interference probe (one GPU): what rank 0's compute loses while it receives the dp
workload's N=8 gather.

At 8 GPUs x 128 images per step, rank 0 receives 7 x 128 x 173 KB = 155 MB of outputs per step from
its peers (the reference's MPI_Gatherv to the root, final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:
125-130; here per-lane RCCL sends). On the receiver that traffic costs HBM bandwidth and the CUs of
the collective's receive channels (RCCL's Simple protocol copies from its FIFO into the user buffer).
One GPU cannot receive over xGMI, so the probe reproduces the receiver-side work: every bench step
(the dp step: 2 free-running lanes of the fp32 Blocks 1-2 engine over rotated inputs) a side stream
copies `--mb` MB into a y_global-sized buffer on exactly W workgroups (anx_channel_copy), W = the
receive channels' CUs. Arms are interleaved in rounds in one process; medians are reported.

Output (stdout, one JSON line per arm + a summary line): ms per step with / without the copy, the
slowdown, the copy's own time and rate (it must move 155 MB within a step, >= 304 GB/s at 0.51 ms,
or the gather cannot keep up regardless). The cost model takes ``ingest_slowdown`` from the arm
that sustains that rate with the fewest workgroups (anx/cost.hpp; profiles/r04_probe_ingest.jsonl).
"""
import argparse
import json
import os
import statistics
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from anx import _native as nat  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--mb", type=float, default=155.06)  # 7 peers x 128 images x 173,056 B
    ap.add_argument("--wgs", default="8,16,32,64,-1", help="workgroups of the copy; -1 = torch copy_ (blit)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = AlexNetBlocks(init="rand", seed=1, device=dev, max_batch=a.batch, lanes=a.lanes)
    g = torch.Generator(device=dev).manual_seed(1)
    xs = [torch.rand((a.batch, 227, 227, 3), device=dev, generator=g) * 0.1 for _ in range(4)]
    y = torch.empty(m.out_shape(a.batch), device=dev)
    nbytes = int(a.mb * 1e6) // 16 * 16
    src = torch.rand(nbytes // 4, device=dev, generator=g)
    dst = torch.empty_like(src)
    side = torch.cuda.Stream(dev)
    wgs = [int(w) for w in a.wgs.split(",")]

    def ingest(wg):
        with torch.cuda.stream(side):
            if wg < 0:
                dst.copy_(src)
            else:
                nat.call("anx_channel_copy", dst.data_ptr(), src.data_ptr(), nbytes, wg, nat.stream_ptr(dev))

    def run(wg, steps):  # ms per step of the bench step with (wg != 0) / without the concurrent ingest
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            m.forward_async(xs[i % len(xs)], y)
            if wg:
                ingest(wg)
        m.join()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / steps

    def copy_alone(wg, reps=10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ingest(wg)
        side.synchronize()
        return (time.perf_counter() - t0) * 1e3 / reps

    t_end = time.perf_counter() + 1.0  # clock settle
    while time.perf_counter() < t_end:
        run(0, 20)
    base, arms, alone = [], {w: [] for w in wgs}, {w: [] for w in wgs}
    for _ in range(a.rounds):
        base.append(run(0, a.steps))
        for w in wgs:
            arms[w].append(run(w, a.steps))
            alone[w].append(copy_alone(w))
    b = statistics.median(base)
    rows = []
    for w in wgs:
        t, c = statistics.median(arms[w]), statistics.median(alone[w])
        rows.append({"probe": "ingest", "workgroups": w, "mb_per_step": round(nbytes / 1e6, 2),
                     "ms_per_step_base": round(b, 4), "ms_per_step_ingest": round(t, 4),
                     "slowdown": round(t / b - 1, 4), "copy_alone_ms": round(c, 4),
                     "copy_gbps": round(nbytes / (c * 1e6), 1), "batch": a.batch, "lanes": a.lanes})
        print(json.dumps(rows[-1]), flush=True)
    need = nbytes / (b * 1e6)  # GB/s the receive side must sustain to keep up with one step
    ok = [r for r in rows if r["workgroups"] > 0 and r["copy_gbps"] >= need]
    pick = min(ok, key=lambda r: r["workgroups"]) if ok else max(rows, key=lambda r: r["copy_gbps"])
    print(json.dumps({"probe": "ingest_summary", "needed_gbps": round(need, 1), "chosen_workgroups": pick["workgroups"],
                      "ingest_slowdown": pick["slowdown"], "base_ms": round(b, 4)}), flush=True)


if __name__ == "__main__":
    main()
