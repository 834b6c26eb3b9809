#!/usr/bin/env python3
"""Headline benchmark: AlexNet Blocks 1-2 fp32 inference throughput (images/s) on N MI355X.

Metric/config from BASELINE.json: "images/sec (and ms/batch) AlexNet Blocks1-2 fp32 at 1/2/4/8
MI355X". One step = every rank runs the native Blocks 1-2 engine (polyphase-Winograd Conv1 and Winograd
Conv2 on f32 MFMA, fused epilogues, pool/LRN kernels) on its own shard of the batch and the outputs
are gathered to rank 0 over RCCL/xGMI (overlapped with the next step's compute). Data-parallel weak
scaling: --batch-per-gpu images per GPU, generated on each rank (--input-source local, the default).
--input-source root reproduces the reference's V4/V5 data flow instead: rank 0 owns the whole batch
and scatters it every step (prefetched one step ahead); that moves 79 MB per peer per 128 images
over xGMI, which binds before the compute does, so it is not the throughput configuration.

The default 600 images per GPU run as 2 lanes of 300 (--lanes: one engine per concurrent HIP stream,
AlexNetBlocks(lanes=...)). 300 per lane is chosen for wave quantization, not memory: both Winograd
GEMMs then launch whole numbers of 512-workgroup waves (1520 and 2544 workgroups), where 128 images
leave a 27 % / 30 % tail round (tools/sweep_batch.py: 128 -> 173k, 300 -> 206k images/s); the second
lane fills the other's tail waves (profiles/r01_ab_lanes_batch.jsonl: 300 x 1 lane 214k, 300 as
2 x 150 217k, 600 as 2 x 300 226k images/s).

Launch: ``python bench.py`` (1 GPU) or ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N``. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import anx  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402
from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather  # noqa: E402

METRIC = "images/sec (and ms/batch) AlexNet Blocks1-2 fp32 at 1/2/4/8 MI355X; speedup+efficiency vs np"
# V3 CUDA single GPU, RTX 3090, 610.661 ms for one image.
BASELINE_IMG_PER_S = 1000.0 / 610.661


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="images per GPU (default 600 for blocks; 256 for full = BASELINE's 2048 over 8 GPUs)")
    # The whole per-rank batch is one launch (fewer, larger launches fill the 256 CUs better); with
    # --no-prefetch, --micro 2 overlaps the second half's scatter with the first half's compute.
    ap.add_argument("--micro", type=int, default=1, help="micro-batches per step for scatter/compute/gather overlap")
    ap.add_argument("--no-prefetch", action="store_true", help="scatter each step's input inside that step only")
    ap.add_argument("--impl", default="mfma", choices=["mfma", "direct"])
    ap.add_argument("--lanes", type=int, default=2,
                    help="concurrent HIP streams per GPU the batch is split over (one engine each)")
    ap.add_argument("--input-source", default="local", choices=["root", "local"],
                    help="local: per-rank synthetic shard (data-parallel); root: rank 0 scatters the batch (V4/V5)")
    ap.add_argument("--no-gather", action="store_true", help="leave outputs on their ranks")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"], help="cpu = gloo rehearsal (tests only)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1-GPU step as one captured HIP graph replayed each step: 1 on, 0 off (default; "
                         "measured equal to eager launches at 300 images, the step is GPU-bound), -1 auto")
    ap.add_argument("--model", default="blocks", choices=["blocks", "full"],
                    help="blocks = the headline AlexNet Blocks1-2 fp32; full = full AlexNet bf16 extension")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=300))  # a hung collective fails in 5 min, not 10
    else:  # CPU rehearsal of the same pipeline over gloo (tests; no GPU)
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo", timeout=timedelta(seconds=300))

    B = a.batch_per_gpu or (256 if a.model == "full" else 600)
    d = anx.blocks_dims()
    if a.model == "full":  # extension config: full AlexNet bf16 (BASELINE.json config 5)
        from anx.models.alexnet_full import FLOPS_PER_IMAGE, AlexNetFull
        model = AlexNetFull(seed=1234, device=dev, max_batch=B)
        out_shape, flops = (1000,), FLOPS_PER_IMAGE
    else:
        model = AlexNetBlocks(init="rand", seed=1234, device=dev, impl=a.impl, max_batch=B, lanes=a.lanes)
        out_shape, flops = (d.Hp2, d.Wp2, d.C2), anx.flops_per_image()
    cfg = PipelineConfig(B, micro=a.micro, scatter=(a.input_source == "root"), gather=not a.no_gather,
                         prefetch=not a.no_prefetch)
    pipe = ScatterComputeGather(model, cfg, (d.H, d.W, d.C0), out_shape, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    if pipe.x_global is not None:
        pipe.x_global.copy_(torch.rand(pipe.x_global.shape, device=dev, generator=g) * 0.1)
    else:  # every input buffer of the (double-buffered) pipeline holds real images
        for xb in pipe._xb:
            xb.copy_(torch.rand(xb.shape, device=dev, generator=g) * 0.1)
    step = pipe.step
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    use_graph = a.graph if a.graph >= 0 else int(world == 1 and dev.type == "cuda")
    if use_graph and world == 1 and dev.type == "cuda":
        # The engine is stream-ordered (no allocation, copy or sync inside a forward), so one step
        # captures as a graph of its kernel launches; a replay then costs one host call per step.
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # first calls pack weights / set kernel attributes outside the capture
                step()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        step = graph.replay

    for _ in range(a.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64 if dev.type == "cuda" else torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el * 1e3 / a.steps
    imgs = B * world * a.steps / el
    if rank == 0 and a.model == "full":
        rec = {
            "metric": "images/sec full AlexNet (Conv1-5 + FC6-8) bf16 inference on MI355X (extension)",
            "value": round(imgs, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic (random images 227x227x3, He-uniform random weights)",
            "config": {"model": "AlexNet full (reference Blocks1-2 + Conv3-5 + FC6-8, 1000 classes)",
                       "global_batch": B * world, "seq_len": None, "parallelism": f"dp{world}",
                       "gflop_per_image": round(flops / 1e9, 4), "tflops": round(imgs * flops / 1e12, 2)},
        }
        print(json.dumps(rec), flush=True)
    elif rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(imgs, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(imgs / BASELINE_IMG_PER_S, 2),
            "dtype": "fp32",
            "data": ("synthetic (U[0,0.1) images 227x227x3 generated on %s, random-init weights)"
                     % ("each rank" if a.input_source == "local" else "rank 0, scattered")),
            "config": {
                "model": "AlexNet Blocks1-2 (Conv1 11x11s4-ReLU-Pool3s2-Conv2 5x5p2-ReLU-Pool3s2-LRN5)",
                "global_batch": B * world,
                "seq_len": None,
                "image": [d.H, d.W, d.C0],
                "parallelism": f"dp{world}",
                "pipeline": (("root scatter -> compute -> gather (RCCL), %d micro-batches%s"
                              % (len(pipe.splits), ", next-step scatter overlapped" if pipe.prefetch else ""))
                             if a.input_source == "root" else
                             "per-rank data -> compute -> gather to rank 0 (RCCL, overlapped with the next step)")
                if world > 1 else "single GPU",
                "input_source": a.input_source,
                "impl": a.impl,
                "lanes": a.lanes,
                "hip_graph": bool(use_graph and world == 1 and dev.type == "cuda"),
                "gflop_per_image": round(anx.flops_per_image() / 1e9, 4),
                "tflops": round(imgs * anx.flops_per_image() / 1e12, 2),
                "ms_per_batch": round(ms, 4),
            },
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
