#!/usr/bin/env python3
"""Headline benchmark: AlexNet Blocks 1-2 fp32 inference throughput (images/s) on N MI355X.

Metric/config from BASELINE.json: "images/sec (and ms/batch) AlexNet Blocks1-2 fp32 at 1/2/4/8
MI355X". Workloads (--workload):

* ``dp`` (default): data-parallel weak scaling. Every rank runs the native Blocks 1-2 engine
  (polyphase-Winograd Conv1 and Winograd Conv2 on exact-fp32 MFMA, fused epilogues, pool/LRN
  kernels) on its own --batch-per-gpu synthetic images; the outputs are gathered to rank 0 over
  RCCL/xGMI, overlapped with the next step's compute. The default per-GPU batch is 128, the
  BASELINE's V5 config per GPU (1024 images over 8 GPUs), run as 2 stream lanes of 64.
* ``v4``: BASELINE config "V4 scatter+halo, batch 256": strong scaling of a fixed global batch that
  starts and ends in host memory — the reference's program shape
  (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:52-130) — run by the native V4 runtime
  (anx/v4.hpp): the batch lives in one shared pinned host segment, every rank DMAs its own images x
  input rows (halo included) over its own host link and its output rows back, in image chunks so
  H2D, compute and D2H overlap. The JSON reports the H2D GB/s in the step and the link's H2D-only
  rate (``h2d_bound_img_s``: what the H2D stage alone would allow).
* ``v5``: BASELINE config "V5 GPU-aware, batch 1024", device-resident "halo + gather": with
  ``--input-source local`` (default) every rank's images x input rows are placed on its device once,
  so a step moves only the per-layer pool1 halos of a row group and the gather (``root``: the
  reference's data flow, the root scatters the batch every step). Run by the native V5 runtime
  (anx/v5.hpp through libanx_dist: halo chunks pipelined against stage1, halo-free ranks as
  free-running stream lanes, the gather of one step on a second stream under the next step's compute,
  weights broadcast device to device). --transport auto | rccl (one GPU per rank) | peer / loopback
  (ranks may share a GPU); --decomp auto (default: the cost model's pick, anx/cost.hpp) | rows (the
  reference's row split over every rank) | hybrid (batch first, rows only below one image per rank) |
  batch.

Every workload's JSON carries a top-level ``model_curve``: the MODELLED 1/2/4/8-GPU curve of its
configuration (``"measured": false``; anx.parallel.cost), with this run's measured single-GPU rate in the
model's throughput table when N = 1. It is kept out of ``config`` so no modelled number sits among the
measured ones.

The dp run also carries ``v4`` and ``v5``: BASELINE configs 3 and 4 (the reference's multi-GPU programs)
measured on the same ranks by the native runtimes, V5 with and without the pool1 halo exchange
(:func:`reference_programs`; ``--no-ref-programs`` skips them).

Launch: ``python bench.py`` (1 GPU) or ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N``. Rank 0 prints ONE JSON line.

Inputs: the dp workload streams ``input_batches_rotated`` distinct synthetic batches (>= 4 and
> 256 MB together, more than the 256 MB Infinity Cache) round-robin through the timed steps.

The reference's own configuration, one image (batch 1) through H2D + forward + D2H, is measured
three ways: ``b1_process_cold_ms`` = a fresh ``anx --version v3`` process (context creation,
allocation, weight upload, copies: what the reference's 610.661 ms timed) started
before this process touches the GPU; ``b1_engine_cold_ms`` = a fresh engine on this already
initialised device (the first of three fresh engines; all three in ``b1_engine_cold_trials_ms``); ``b1_warm_ms`` = the median of further calls. ``vs_baseline`` is the
like-for-like cold ratio 610.661 ms / ``b1_process_cold_ms`` (``vs_baseline_kind`` says which ratio
it is); the warm ratio is ``b1_vs_reference_warm``. ``mfma_tflops`` counts the matrix-core FLOPs the Winograd
kernels execute (0.237 GFLOP/image with 4x4-tile Conv2); ``direct_equiv_tflops`` counts direct-convolution FLOPs
(1.107 GFLOP/image) and can exceed the chip's fp32 peak because Winograd does 4x fewer multiplies.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues round-robin (4 on the MI355X boxes). Two
# lanes' streams on one queue serialise (0.80 vs 0.57 ms per 128-image step when other streams were
# created first: profiles/r02_lanes_async.txt); 8 gives every stream here (current, 2 lanes, RCCL) its
# own. Read by the HIP runtime at its first call, so set before torch touches the GPU (the boxes
# export 4 explicitly; ANX_HW_QUEUES overrides the 8).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ANX_HW_QUEUES", "8")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import anx  # noqa: E402
from anx.config import mfma_flops_per_image  # noqa: E402
from anx.models.alexnet_blocks import AlexNetBlocks  # noqa: E402
from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather  # noqa: E402

METRIC = "images/sec (and ms/batch) AlexNet Blocks1-2 fp32 at 1/2/4/8 MI355X; speedup+efficiency vs np"
BASELINE_V3_MS = 610.661  # V3 CUDA single GPU, RTX 3090, one image, cold
MODEL = "AlexNet Blocks1-2 (Conv1 11x11s4-ReLU-Pool3s2-Conv2 5x5p2-ReLU-Pool3s2-LRN5)"
DEFAULT_BATCH = {"dp": 128, "v4": 256, "v5": 1024}


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="dp", choices=["dp", "v4", "v5"])
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="dp: images per GPU (default 128 for blocks; 256 for full = BASELINE's 2048 over 8 GPUs)")
    ap.add_argument("--batch", type=int, default=None, help="v4/v5: global batch (default 256 / 1024)")
    ap.add_argument("--decomp", default=None, choices=["auto", "rows", "hybrid", "batch"],
                    help="v4/v5 decomposition (default on GPU: auto = the cost model's pick; rows on the CPU rehearsal)")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "peer", "loopback"],
                    help="v5 device transport")
    ap.add_argument("--chunks", type=int, default=0, help="v5: halo pipeline chunks per step (0 = auto)")
    ap.add_argument("--pipeline", type=int, default=-1, choices=[-1, 0, 1],
                    help="v5: next-step scatter / this-step gather on a second stream (-1 auto)")
    ap.add_argument("--micro", type=int, default=1, help="dp: micro-batches per step for scatter/compute/gather overlap")
    ap.add_argument("--no-prefetch", action="store_true", help="dp: scatter each step's input inside that step only")
    ap.add_argument("--impl", default="mfma", choices=["mfma", "direct"])
    ap.add_argument("--lanes", type=int, default=2,
                    help="concurrent HIP streams per GPU the batch is split over (one engine each)")
    ap.add_argument("--full-lanes", type=int, default=1,
                    help="--model full: concurrent stream lanes the batch is split over (AlexNetFull lanes)")
    ap.add_argument("--input-source", default="local", choices=["root", "local"],
                    help="dp / v5: local = per-rank (device-resident) data; root = rank 0 scatters the batch every step")
    ap.add_argument("--no-gather", action="store_true", help="dp: leave outputs on their ranks")
    ap.add_argument("--root-batch", type=int, default=-1,
                    help="dp, local input, N>1: images rank 0 computes per step while it also receives the gather "
                         "(-1 = the cost model's shed share on GPUs / off on the CPU rehearsal, 0 = off, >0 = that many)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"], help="cpu = gloo rehearsal (tests only)")
    ap.add_argument("--graph", type=int, default=0,
                    help="dp, 1 GPU: the step as one captured HIP graph replayed each step (1; joins the lanes per "
                         "step: 231-236 k vs 322-323 k images/s free-running, profiles/r05_knob_ab/), eager (0, "
                         "default), -1 auto")
    ap.add_argument("--no-b1", action="store_true", help="skip the batch-1 latency measurement")
    ap.add_argument("--lane-priority", type=int, default=0, help="dp: HIP stream priority of the side lanes (-1 = high)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="blocks model: engine knob override (anx.utils.tuning.KNOBS), repeatable; A/B only")
    ap.add_argument("--stagger", action="store_true",
                    help="dp: free-running lanes restart half a forward apart after a device sync (default: together)")
    ap.add_argument("--joined-lanes", action="store_true",
                    help="dp: join the stream lanes every step (AlexNetBlocks.forward) instead of free-running lanes "
                         "half a step apart (forward_async; the default with local input)")
    ap.add_argument("--prewarm-s", type=float, default=1.0,
                    help="GPU: seconds of untimed steps before the warmup steps, so the timed steps run at the "
                         "loaded clock (0 = off)")
    ap.add_argument("--model", default="blocks", choices=["blocks", "full"],
                    help="blocks = the headline AlexNet Blocks1-2 fp32; full = full AlexNet bf16 extension")
    ap.add_argument("--calibrate-root", default="auto", choices=["auto", "on", "off"],
                    help="dp, N>1 with root shedding: measure per-rank compute spans before the warmup and rescale "
                         "rank 0's share to the peers' (auto = on when the share is the cost model's, not --root-batch)")
    ap.add_argument("--no-verify", action="store_true",
                    help="dp, N>1: skip the post-window gather checksum / oracle verification step")
    ap.add_argument("--no-subrecords", action="store_true",
                    help="v5: skip the forced 2-way-row (halo on) sub-records per device transport")
    ap.add_argument("--no-ref-programs", action="store_true",
                    help="dp: skip the V4 / V5 secondary records (BASELINE configs 3 and 4) beside the headline")
    ap.add_argument("--ref-steps", type=int, default=5, help="timed steps of each V4 / V5 secondary arm")
    ap.add_argument("--ref-batch-v4", type=int, default=2, help="CPU rehearsal only: V4 secondary global batch")
    ap.add_argument("--ref-batch-v5", type=int, default=3, help="CPU rehearsal only: V5 secondary global batch")
    ap.add_argument("--no-full", action="store_true",
                    help="blocks dp on GPUs: skip the secondary full-AlexNet bf16 (BASELINE config 5) measurement")
    ap.add_argument("--first-collective-s", type=float, default=float(os.environ.get("ANX_FIRST_COLLECTIVE_S", "240")),
                    help="N>1: seconds the process-group setup and first collectives may take before the rank exits "
                         "with a rank-tagged error (0 = no watchdog)")
    ap.add_argument("--cold-gap-s", type=float, default=2.0,
                    help="seconds between the fresh-process batch-1 children (a HIP start-up right after another "
                         "GPU process exits waits for that process's teardown)")
    ap.add_argument("--cold-trials", type=int, default=3,
                    help="fresh anx v3 processes for the cold batch-1 record (the median is reported)")
    ap.add_argument("--secondary-deadline-s", type=float,
                    default=float(os.environ.get("ANX_SECONDARY_DEADLINE_S", "150")),
                    help="seconds the secondary records (batch-1 probes, native V4/V5 programs, bf16 extension) and "
                         "the closing barrier may take after the headline is measured; past it rank 0 prints the "
                         "headline with the pending secondaries marked and every rank exits 0 (0 = no deadline)")
    return ap.parse_args()


def process_cold_b1(gap_s: float = 2.0, trials: int = 3) -> dict:
    """The reference's V3 timing, like for like: one image through a FRESH process (`anx --version v3`:
    context creation, allocations, weight upload, H2D, forward, D2H), started before this process
    touches the GPU. The child gets a single-process environment (no torchrun rank variables).

    Each child starts `gap_s` after the previous GPU process ended: a HIP process started right after
    another one exits spends 160-225 ms in hipInit (the driver is still tearing the previous process down)
    against ~50 ms after a 2 s gap (profiles/r06_cold/gap.log), so back to back the probes would time
    each other's teardown, not the runtime's start-up. The child runs `trials` times (fresh processes, gaps
    between): the record is the median trial, every trial's cold_ms listed (the shared host's other GPU
    processes still stall a start-up now and then: 81 vs 219 ms init in two runs of the same tree)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cuda-mpi-gpu-cluster-programming_amd", "bin", "anx")
    if not os.path.exists(exe):
        return {"b1_process_cold_ms": None, "b1_process_note": "native CLI not built"}
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ANX_RANK", "ANX_WORLD_SIZE", "ANX_LOCAL_RANK")}
    probe = os.path.join(os.path.dirname(exe), "anx_hipinit")

    def bare():  # the bare HIP runtime's start-up in a fresh process without libanx (anx_hipinit)
        if not os.path.exists(probe):
            return None
        try:
            p = subprocess.run([probe, "pinned"], capture_output=True, text=True, timeout=120, env=env)
            js = [json.loads(l[len("ANX_JSON "):]) for l in p.stdout.splitlines() if l.startswith("ANX_JSON ")]
            return js[0] if p.returncode == 0 and js else None
        except Exception:
            return None

    time.sleep(gap_s)  # a GPU process (e.g. the driver's smoke run) may have just ended
    bare0 = bare()
    runs = []  # (record, wall ms) per fresh anx child
    for _ in range(max(1, trials)):
        time.sleep(gap_s)
        t0 = time.perf_counter()
        out = subprocess.run([exe, "--version", "v3", "--batch", "1", "--init", "rand", "--iters", "20"],
                             capture_output=True, text=True, timeout=300, env=env)
        wall = (time.perf_counter() - t0) * 1e3
        recs = [json.loads(l[len("ANX_JSON "):]) for l in out.stdout.splitlines() if l.startswith("ANX_JSON ")]
        if out.returncode != 0 or not recs:
            return {"b1_process_cold_ms": None, "b1_process_note": f"anx v3 failed rc={out.returncode}"}
        runs.append((recs[0], wall))
    time.sleep(gap_s)
    bare1 = bare()
    r, wall = sorted(runs, key=lambda rw: rw[0]["cold_ms"])[len(runs) // 2]  # the median trial
    # the same steps as the anx child's `init` phase (hipInit .. first stream), timed in a process that does
    # not load libanx, once before and once after the anx child: what the HIP runtime costs by itself
    binit = [round(b["hip_init_ms"] + b["device_count_ms"] + b["context_ms"] + b["stream_ms"], 3)
             for b in (bare0, bare1) if b]
    ph = {k: round(v, 3) for k, v in (r.get("phases_cold") or {}).items()}
    init_split = {}
    if binit and "init" in ph:
        init_split = {"init_bare_hip_ms": binit, "init_ours_ms": round(ph["init"] - min(binit), 3),
                      "init_note": "init_bare_hip_ms: anx_hipinit (no libanx) before the first / after the last "
                                   "anx child; init_ours_ms = the median child's init minus the faster bare probe "
                                   "(a start-up right after another GPU process exits takes 160-225 ms instead of "
                                   "~50: profiles/r06_cold/gap.log)"}
    return {"b1_process_cold_ms": round(r["cold_ms"], 3), "b1_process_wall_ms": round(wall, 1),
            "b1_process_cold_trials_ms": [round(x["cold_ms"], 3) for x, _ in runs], **init_split,
            # where the cold time goes (init = HIP runtime / context, engine = weights + workspace, alloc,
            # h2d / compute / d2h of the first image)
            "b1_process_phases_ms": ph,
            "b1_process_warm_ms": round(float(r["warm_ms"]), 4),
            "b1_process_cold_vs_reference": round(BASELINE_V3_MS / r["cold_ms"], 2),
            "b1_process_note": "anx --version v3 --batch 1 child: cold_ms from main() entry incl. HIP context "
                               "creation; wall_ms incl. exec, library load and teardown; the median of "
                               "b1_process_cold_trials_ms (fresh processes, each started b1_process_gap_s after "
                               "the previous GPU process ended)",
            "b1_process_gap_s": gap_s}


def batch1_latency(dev, reps: int = 20) -> dict:
    """The reference's V3 configuration (v3_cuda_only/src/main_cuda.cpp:30-35): one image, timed
    around H2D + forward + D2H. cold = a fresh engine (allocation, weight upload, first launch) on
    an already-initialised device; warm = median of `reps` further calls."""
    from anx.utils.init import init_weights
    x = (torch.rand(1, 227, 227, 3) * 0.1).pin_memory()
    w = init_weights("rand", 7)  # host weights exist before the clock starts (the reference's V3 fills them
    colds = []                    # on the host before its timed region too)
    for _ in range(3):  # three fresh engines (each its own allocations, uploads and first launch); the
        torch.cuda.synchronize()  # first is the record (later ones reuse freed device memory), all are reported
        t0 = time.perf_counter()
        m = AlexNetBlocks(w, device=dev, max_batch=1)
        y = m(x.to(dev, non_blocking=True)).cpu()
        colds.append((time.perf_counter() - t0) * 1e3)
        if len(colds) < 3:
            m.close()
    cold = colds[0]
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        y = m(x.to(dev, non_blocking=True)).cpu()
        ts.append((time.perf_counter() - t0) * 1e3)
    del y
    m.close()
    warm = sorted(ts)[len(ts) // 2]
    return {"b1_engine_cold_ms": round(cold, 3), "b1_engine_cold_trials_ms": [round(c, 3) for c in colds],
            "b1_warm_ms": round(warm, 4),
            "b1_engine_cold_vs_reference": round(BASELINE_V3_MS / cold, 1),
            "b1_vs_reference_warm": round(BASELINE_V3_MS / warm, 1)}


def full_bf16_secondary(dev, world: int, rank: int, steps: int = 10, warmup: int = 3, prewarm_s: float = 0.5) -> dict:
    """BASELINE config 5 beside the headline: full AlexNet (Conv1-5 + FC6-8) bf16, 256 images per GPU,
    weak scaling (each rank its own batch, no gather), timed like the headline over a short window."""
    from anx.models.alexnet_full import FLOPS_PER_IMAGE, AlexNetFull
    B = 256
    m = AlexNetFull(seed=1234, device=dev, max_batch=B)
    g = torch.Generator(device=dev)
    g.manual_seed(77 + rank)
    xs = [torch.rand((B, 227, 227, 3), device=dev, generator=g) for _ in range(2)]
    y = torch.empty((B, 1000), device=dev)
    k = 0
    t0 = time.perf_counter()
    while True:  # clock settle (also the first-call setup)
        for _ in range(8):
            m(xs[k % 2], y)
            k += 1
        torch.cuda.synchronize()
        if time.perf_counter() - t0 > prewarm_s:
            break
    for _ in range(warmup):
        m(xs[k % 2], y)
        k += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m(xs[k % 2], y)
        k += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    finite = bool(torch.isfinite(y).all().item())
    m.close()
    ips = B * world * steps / el
    return {"metric": "images/sec full AlexNet (Conv1-5 + FC6-8) bf16 inference (BASELINE config 5, extension)",
            "value": round(ips, 1), "unit": "images/s", "ms_per_step": round(el * 1e3 / steps, 4), "steps": steps,
            "warmup": warmup, "batch_per_gpu": B, "global_batch": B * world, "n_gpus": world, "dtype": "bf16",
            "scaling": "weak", "tflops": round(ips * FLOPS_PER_IMAGE / 1e12, 1), "outputs_finite": finite,
            "data": "synthetic images, He-uniform random weights", "note": "secondary record; the headline is fp32"}


def v5_halo_subrecords(a, world: int, rank: int, GB: int, dev, g) -> dict:
    """BASELINE config 4 with the per-layer halo exchange forced on: 2-way row groups (the pool1 halo
    between the two ranks of a group moves every step), once per device transport, so a run measures
    RCCL against the peer (IPC copy + device flag) transport side by side with the halo bytes and the
    halo_p1 wait. One GPU: two ranks sharing it as child processes (`anxrun -np 2 anx --version v5`;
    peer, and the RCCL transport's code over the loopback device comm, since RCCL refuses a shared
    device). N > 1 (even): in process, every rank."""
    import subprocess
    out = {}
    if world == 1:
        if rank != 0:
            return out
        root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cuda-mpi-gpu-cluster-programming_amd", "bin")
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
        for tr in ("peer", "loopback"):
            cmd = [os.path.join(root, "anxrun"), "-np", "2", "--timeout", "200", "--", os.path.join(root, "anx"),
                   "--version", "v5", "--transport", tr, "--batch", str(GB), "--row-ways", "2", "--iters", "10",
                   "--init", "rand", "--chunks", "1"]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
                recs = [json.loads(l[len("ANX_JSON "):]) for l in r.stdout.splitlines() if l.startswith("ANX_JSON ")]
                if r.returncode != 0 or not recs:
                    out[f"v5_rows2_{tr}"] = {"error": f"rc={r.returncode}", "stderr": r.stderr[-300:]}
                    continue
                j = recs[0]
                v5 = j.get("v5") or {}
                out[f"v5_rows2_{tr}"] = {
                    "ranks": 2, "shared_gpu": True, "row_ways": 2, "transport": v5.get("transport", tr),
                    "images_per_s": float(j["images_per_s"]) if j.get("images_per_s") not in (None, "null") else None,
                    "ms_per_step": float(j["warm_ms"]) if j.get("warm_ms") not in (None, "null") else None,
                    "phases_ms": j.get("phases_warm"), "halo_exchange": v5.get("halo_exchange"),
                    "halo_bytes_per_step": v5.get("halo_bytes_per_step"),
                    "bytes_per_step": v5.get("bytes_per_step"), "checksum": j.get("checksum")}
            except Exception as e:  # a sub-record never takes the headline down
                out[f"v5_rows2_{tr}"] = {"error": repr(e)[:300]}
        _match_arms(out, "loopback", "peer", "checksum")
        return out
    if world % 2:
        return out
    from anx.parallel import selfcheck
    from anx.parallel.workloads import NativeV5
    from anx.utils.init import init_weights
    b1, b2 = anx.config.blocks()
    for tr in ("rccl", "peer"):
        wl = NativeV5(GB, init_weights("rand", 1234, b1, b2) if rank == 0 else None, specs=(b1, b2), decomp="rows2",
                      transport=tr, chunks=a.chunks, pipeline=a.pipeline, impl=a.impl, input_source="local",
                      lanes=a.lanes)
        wl.fill((torch.rand((GB, 227, 227, 3), device=dev, generator=g) * 0.1) if rank == 0 else None)
        wl.step(steps=3)
        wl.sync()
        wl.reset_phases()
        dist.barrier()
        t0 = time.perf_counter()
        wl.step(steps=10)
        wl.sync()
        dist.barrier()
        el = time.perf_counter() - t0
        d = wl.describe()
        y = wl.output()  # rank 0: the gathered output of the last step (both transports: identical math)
        out[f"v5_rows2_{tr}"] = {"ranks": world, "row_ways": 2, "transport": d.get("transport"),
                                 "images_per_s": round(GB * 10 / el, 1), "ms_per_step": round(el * 100, 4),
                                 "phases_ms": wl.phase_ms(), "halo_exchange": d.get("halo_exchange"),
                                 "halo_bytes_per_step": d.get("halo_bytes_per_step"),
                                 "bytes_per_step": d.get("bytes_per_step"),
                                 "output_crc": selfcheck.tensor_crc(y) if y is not None else None}
        wl.close()
    _match_arms(out, "rccl", "peer", "output_crc")
    return out


def _native_arm(wl, GB: int, world: int, rank: int, steps: int, warmup: int, dev) -> dict:
    """Time one native V4 / V5 runtime (warmup, then ``steps`` timed steps bracketed by a barrier and a
    sync, max over ranks) and describe it: rate, halo exchange and bytes, phases, exact output checksum."""
    from anx.parallel import selfcheck
    wl.step(steps=warmup)
    wl.sync()
    wl.reset_phases()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    wl.step(steps=steps)
    wl.sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    d, ph = wl.describe(), wl.phase_ms()
    y = wl.output()
    rec = {"global_batch": GB, "n_gpus": world, "steps": steps, "images_per_s": round(GB * steps / el, 1),
           "ms_per_step": round(el * 1e3 / steps, 4), "row_ways": d.get("row_ways"),
           "halo_exchange": d.get("halo_exchange"), "phases_ms": ph, "halo_p1_ms": ph.get("halo_p1")}
    for k in ("transport", "decomp", "halo_bytes_per_step", "halo_transfers_per_step", "input_source", "lanes",
              "h2d_bytes_per_step_rank", "staging"):
        if k in d:
            rec[k] = d[k]
    if y is not None:
        rec["output_crc"] = selfcheck.tensor_crc(y)
    return rec


def reference_programs(a, world: int, rank: int, dev, cuda: bool, g) -> dict:
    """BASELINE configs 3 and 4 beside the dp headline, on the same ranks: the reference's
    multi-GPU programs, V4 (256 images, host-staged scatter + per-rank rows) and V5 (1024 images,
    device-resident, per-layer pool1 halo + gather), run by the native runtimes (anx/v4.hpp, anx/v5.hpp),
    strong scaling. V5 runs twice: the cost model's pick (``auto``: usually a batch split, no halo) and a
    forced row split with the halo exchange ON (``rows2``: 2-way row groups; ``rows`` at an odd rank count),
    the latter once per device transport (RCCL, and the peer IPC transport at N > 1) with matching exact
    checksums. At N = 1 the forced-halo arms are two ranks sharing the GPU (v5_halo_subrecords). CPU ranks
    (tests) run the V5 runtime in host mode on a few images. Every arm sits in its own try/except: the
    headline never depends on them."""
    from anx.parallel.workloads import NativeV4, NativeV5
    from anx.utils.init import init_weights
    b1s, b2s = anx.config.blocks()
    d = anx.blocks_dims()
    w = init_weights("rand", 1234, b1s, b2s) if rank == 0 else None
    gb4, gb5 = (a.ref_batch_v4, a.ref_batch_v5) if not cuda else (256, 1024)
    steps, warm = (a.ref_steps, 1) if not cuda else (a.ref_steps, 2)
    out = {"v4": {}, "v5": {}}

    def batch_x(GB):
        if rank != 0:
            return None
        gen = torch.Generator().manual_seed(4321)
        return torch.rand((GB, d.H, d.W, d.C0), generator=gen) * 0.1

    def arm(dst, name, make, GB):
        wl = None
        try:
            wl = make()
            wl.fill(batch_x(GB))
            dst[name] = _native_arm(wl, GB, world, rank, steps, warm, dev)
        except Exception as e:  # a secondary record never takes the headline down
            dst[name] = {"error": repr(e)[:300]}
        finally:
            if wl is not None:
                wl.close()

    # V4 (BASELINE config 3): the runtime's default split
    if cuda:
        arm(out["v4"], "auto", lambda: NativeV4(gb4, w, specs=(b1s, b2s), decomp="auto", impl=a.impl), gb4)
    else:
        arm(out["v4"], "auto", lambda: NativeV5(gb4, w, specs=(b1s, b2s), decomp="auto", impl="host",
                                                input_source="root", layer="overlap"), gb4)
    # V5 (BASELINE config 4): auto, then the halo forced on
    halo = "rows2" if world % 2 == 0 else "rows"
    if cuda:
        arm(out["v5"], "auto", lambda: NativeV5(gb5, w, specs=(b1s, b2s), decomp="auto", impl=a.impl,
                                                input_source="local", lanes=a.lanes), gb5)
        if world > 1:
            for tr in ("rccl", "peer"):
                arm(out["v5"], f"{halo}_{tr}", lambda: NativeV5(gb5, w, specs=(b1s, b2s), decomp=halo, transport=tr,
                                                               impl=a.impl, input_source="local", lanes=a.lanes), gb5)
            _match_arms(out["v5"], f"{halo}_rccl", f"{halo}_peer", "output_crc", prefix="")
        else:
            out["v5"].update({k.replace("v5_", ""): v for k, v in v5_halo_subrecords(a, world, rank, gb5, dev, g).items()})
    else:
        arm(out["v5"], "auto", lambda: NativeV5(gb5, w, specs=(b1s, b2s), decomp="auto", impl="host"), gb5)
        if world > 1:
            arm(out["v5"], f"{halo}_host", lambda: NativeV5(gb5, w, specs=(b1s, b2s), decomp=halo, impl="host"), gb5)
    for k, v in (("v4", "BASELINE config 3: V4 scatter+halo, batch 256 (host-staged; native V4 runtime)"),
                 ("v5", "BASELINE config 4: V5 GPU-aware, batch 1024 (device-resident halo + gather; native V5 "
                        "runtime)")):
        out[k]["config"] = v
        out[k]["scaling"] = "strong"
    return out


def _match_arms(out: dict, a: str, b: str, key: str, prefix: str = "v5_rows2_") -> None:
    """The peer transport's cross-device ordering (flag write after the copy into the receiver's memory)
    checked on the node that runs it: both arms compute the same tiles with the same kernels, so their
    outputs must agree bit for bit; ``outputs_match`` goes into the second arm's record."""
    ra, rb = out.get(f"{prefix}{a}") or {}, out.get(f"{prefix}{b}") or {}
    if ra.get(key) is not None and rb.get(key) is not None:
        rb["outputs_match_" + a] = ra[key] == rb[key]


def _oracle(model):
    """fp64 PyTorch oracle of one image (max |y - ref| / max |ref|)."""
    from anx.models.reference import blocks_forward

    def check(x1, y1):
        ref = blocks_forward(x1.detach().cpu(), model.weights, model.b1, model.b2)
        return float((y1.detach().cpu().double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    return check


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    # before this process's first GPU call (a child of a GPU-initialised process would not be cold)
    b1p = process_cold_b1(a.cold_gap_s, a.cold_trials) if (rank == 0 and a.device == "cuda" and not a.no_b1 and a.model == "blocks") else {}
    from anx.parallel import selfcheck
    ident = None
    with selfcheck.FirstCollectiveWatchdog(rank, a.first_collective_s if world > 1 else 0,
                                           "process-group setup + first collective"):
        if a.device == "cuda":
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
            if world > 1:
                dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=300))  # a hung collective fails in 5 min, not 10
        else:  # CPU rehearsal of the same program over gloo (tests; no GPU)
            dev = torch.device("cpu")
            if world > 1:
                dist.init_process_group("gloo", timeout=timedelta(seconds=300))
        if world > 1:
            ident = selfcheck.rank_identity(dev)  # the first collective: every rank's device, gathered
    cuda = dev.type == "cuda"

    d = anx.blocks_dims()
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    wl = None
    knobs = {k: int(v) if v.lstrip("-").isdigit() else v for k, v in (kv.split("=", 1) for kv in a.knob)}
    if a.model == "full":  # extension config: full AlexNet bf16 (BASELINE.json config 5)
        from anx.models.alexnet_full import FLOPS_PER_IMAGE, AlexNetFull
        B = a.batch_per_gpu or 256
        model = AlexNetFull(seed=1234, device=dev, max_batch=B, lanes=a.full_lanes, knobs=knobs)
        out_shape, flops = (1000,), FLOPS_PER_IMAGE
    elif a.workload == "dp":
        B = a.batch_per_gpu or DEFAULT_BATCH["dp"]
        model = AlexNetBlocks(init="rand", seed=1234, device=dev, impl=a.impl, max_batch=B, lanes=a.lanes,
                              lane_priority=a.lane_priority, knobs=knobs)
        model.stagger = a.stagger
        out_shape, flops = (d.Hp2, d.Wp2, d.C2), anx.flops_per_image()
    else:
        GB = a.batch or DEFAULT_BATCH[a.workload]
        a.decomp = a.decomp or ("auto" if cuda else "rows")
        if a.workload == "v4" and cuda:
            # the native V4 runtime: shared pinned host segment, per-rank chunked DMA (anx/v4.hpp)
            from anx.parallel.workloads import NativeV4
            from anx.utils.init import init_weights
            b1, b2 = anx.config.blocks()
            wl = NativeV4(GB, init_weights("rand", 1234, b1, b2) if rank == 0 else None, specs=(b1, b2),
                          decomp=a.decomp, chunks=a.chunks, impl=a.impl)
            wl.fill((torch.rand((GB, d.H, d.W, d.C0), generator=torch.Generator().manual_seed(1234)) * 0.1)
                    if rank == 0 else None)
        else:
            # the native V5 runtime: plan, buffers, streams and transport live in C++ (anx/v5.hpp). CPU
            # ranks run the same runtime in host mode (host engine + host transport); V4 on CPU is its
            # overlap-tile layer with the batch scattered from the root each step.
            from anx.parallel.workloads import NativeV5
            from anx.utils.init import init_weights
            b1, b2 = anx.config.blocks()
            kw = dict(transport=a.transport, pipeline=a.pipeline, impl=a.impl, input_source=a.input_source,
                      lanes=a.lanes)
            if not cuda:
                kw = dict(impl="host", input_source="root" if a.workload == "v4" else a.input_source,
                          layer="overlap" if a.workload == "v4" else "per_layer")
            wl = NativeV5(GB, init_weights("rand", 1234, b1, b2) if rank == 0 else None, specs=(b1, b2),
                          decomp=a.decomp, chunks=a.chunks, **kw)
            wl.fill((torch.rand((GB, d.H, d.W, d.C0), device=dev, generator=g) * 0.1) if rank == 0 else None)
        step = wl.step
        B = GB  # images per step (whole job)
        out_shape, flops = (d.Hp2, d.Wp2, d.C2), anx.flops_per_image()

    use_graph = False
    root_b, root_note = B, None
    if wl is None and a.model == "blocks" and world > 1 and a.input_source == "local" and not a.no_gather:
        from anx.parallel.pipeline import root_batch_for
        if a.root_batch > 0:
            root_b = min(B, a.root_batch)
        elif a.root_batch < 0 and cuda:
            from anx.parallel import cost
            root_b = cost.dp_root_batch(world, B)
        # never a share that changes the root's lane or micro-batch count (8 x 32 images: 30 -> 32)
        root_b, root_note = root_batch_for(root_b, B, a.micro, getattr(model, "lane_bounds", None))
    if wl is None:
        cfg = PipelineConfig(B, micro=a.micro, scatter=(a.input_source == "root"), gather=not a.no_gather,
                             root_batch=root_b,
                             prefetch=not a.no_prefetch,
                             async_lanes=not a.joined_lanes and a.graph == 0
                             and (a.full_lanes if a.model == "full" else a.lanes) > 1)
        pipe = ScatterComputeGather(model, cfg, (d.H, d.W, d.C0), out_shape, dev)
        if pipe.x_global is not None:
            pipe.x_global.copy_(torch.rand(pipe.x_global.shape, device=dev, generator=g) * 0.1)
        else:  # every input buffer of the (double-buffered) pipeline holds real images
            for xb in pipe._xfull:
                xb.copy_(torch.rand(xb.shape, device=dev, generator=g) * 0.1)
        step = pipe.step
        use_graph = bool(a.graph if a.graph >= 0 else world == 1) and world == 1 and cuda
        if pipe.x_global is None and not use_graph and cuda:
            # distinct batches round-robin: >= 4 and > 256 MB together, so the input is not resident in
            # the 256 MB Infinity Cache (a captured graph replays one input pointer: no rotation there)
            nb = pipe._xfull[0].numel() * 4
            n_rot = min(64, max(4, -(-(300 << 20) // nb)))
            pipe.inputs = [torch.rand(pipe._xfull[0].shape, device=dev, generator=g) * 0.1 for _ in range(n_rot)]
        if use_graph:
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
    sync = torch.cuda.synchronize if cuda else (lambda: None)

    # Clock settle before the W warmup steps: the chip needs ~0.5 s of sustained load to reach its
    # loaded clock (20 steps after 5 warmups measured 0.676 ms/step, 300 steps 0.628, same box:
    # profiles/r02_bench_warmup.txt). Untimed, bounded by --prewarm-s, reported in the JSON.
    # Every rank runs the same number of steps (step() holds collectives): 8 steps (first-call setup),
    # 8 timed probe steps, then as many more as the slowest rank's probe says fill the budget.
    # rank 0's share, measured: per-rank lane compute spans while rank 0 receives (selfcheck)
    calib = None
    calibrate = a.calibrate_root == "on" or (a.calibrate_root == "auto" and a.root_batch < 0)
    if wl is None and world > 1 and pipe.shed and pipe.async_lanes and calibrate:
        from anx.models.alexnet_blocks import LANE_MIN
        for _ in range(4):  # first-call setup outside the measured rounds
            step()
        lanes_b = len(model.lane_bounds(B)) - 1 if hasattr(model, "lane_bounds") else 1
        calib = selfcheck.calibrate_root_batch(pipe, step, torch.cuda.synchronize if cuda else (lambda: None),
                                               min_root=min(B, lanes_b * LANE_MIN if lanes_b > 1 else 1))
        root_b = pipe.root_batch
    t_pw, n_pw = time.perf_counter(), 0
    if cuda and a.prewarm_s > 0:
        for _ in range(8):
            step()
        sync()
        t1 = time.perf_counter()
        for _ in range(8):
            step()
        sync()
        dt = time.perf_counter() - t1
        left = a.prewarm_s - (time.perf_counter() - t_pw)
        if world > 1:
            t = torch.tensor([dt, left], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt, left = float(t[0].item()), float(t[1].item())
        n_pw = 16 + min(50000, int(max(0.0, left) / max(dt, 1e-6) * 8))
        for _ in range(n_pw - 16):
            step()
        sync()
    prewarm_ms = round((time.perf_counter() - t_pw) * 1e3, 1)

    for _ in range(a.warmup):
        step()
    sync()
    if hasattr(wl, "reset_phases"):
        wl.reset_phases()  # the native runtime times every step: keep only the timed ones
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if wl is not None:
        for _ in range(a.steps):
            wl.step(record=True)
    else:
        for _ in range(a.steps):
            step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el * 1e3 / a.steps
    per_step = B if wl is not None else B * (world - 1) + root_b  # images per step over the whole job
    imgs = per_step * a.steps / el
    phases = wl.phase_ms() if wl is not None else None
    # N > 1: one more (untimed) step, then prove the gather and the numerics (selfcheck.verify_gather)
    verify = None
    if wl is None and world > 1 and not a.no_verify and a.model == "blocks":
        step()
        pipe.drain()
        sync()
        corrupt = os.environ.get("ANX_BENCH_CORRUPT_RANK")
        verify = selfcheck.verify_gather(pipe, oracle=_oracle(model),
                                         corrupt_rank=int(corrupt) if corrupt not in (None, "") else None)

    if a.model == "full":
        if rank == 0:
            rec = {
                "metric": "images/sec full AlexNet (Conv1-5 + FC6-8) bf16 inference on MI355X (extension)",
                "value": round(imgs, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "bf16", "data": "synthetic (random images 227x227x3, He-uniform random weights)",
                "config": {"model": "AlexNet full (reference Blocks1-2 + Conv3-5 + FC6-8, 1000 classes)",
                           "global_batch": B * world, "seq_len": None, "parallelism": f"dp{world}",
                           "gflop_per_image": round(flops / 1e9, 4), "tflops": round(imgs * flops / 1e12, 2),
                           "prewarm_steps": n_pw, "prewarm_ms": prewarm_ms, "lanes": a.full_lanes, "knobs": a.knob,
                           "lane_sync": ("free-running lanes, staggered at a mid-forward event (forward_async)" if pipe.async_lanes
                                         else "lanes forked/joined every step" if a.full_lanes > 1 else "one lane")},
            }
            print(json.dumps(rec), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    rec = None
    if rank == 0:  # the headline record, complete before any secondary runs
        from anx.utils.tuning import default_knob
        mf = mfma_flops_per_image(conv2_tile=int(knobs.get("conv2_tile", default_knob("conv2_tile"))))
        if wl is None:
            par, scaling = f"dp{world}", "weak"
            pipeline = (("root scatter -> compute -> gather (RCCL), %d micro-batches%s"
                         % (len(pipe.splits), ", next-step scatter overlapped" if pipe.prefetch else ""))
                        if a.input_source == "root" else
                        "per-rank data -> compute -> gather to rank 0 (RCCL, overlapped with the next step)") \
                if world > 1 else "single GPU"
            rot = pipe.inputs or []
            extra = {"input_source": a.input_source, "lanes": a.lanes, "hip_graph": use_graph, "knobs": a.knob,
                     "batch_per_gpu": B, "root_batch": root_b,
                     **({"root_batch_modelled": cfg.root_batch, **calib} if calib else {}),
                     "root_batch_note": root_note or (("rank 0 sheds the share its gather ingest costs it (cost "
                                                      "model dp_root_batch; tools/probe_ingest.py)")
                                                     if root_b != B else None),
                     "input_batches_rotated": len(rot) or 1,
                     "input_bytes_rotated": sum(t.numel() * 4 for t in rot) or pipe._xb[0].numel() * 4,
                     "lane_sync": ("free-running lanes (%s start), per-lane gathers (forward_async)"
                                   % ("staggered" if a.stagger else "joint")
                                   if pipe.async_lanes else "lanes forked/joined every step")}
        else:
            par, scaling = f"{a.workload}-{a.decomp}{world}", "strong"
            pipeline = ("shared pinned host segment -> per-rank chunked H2D over its own link -> overlap tiles "
                        "-> per-rank D2H into the segment (host-staged, no device collectives)"
                        if a.workload == "v4" and cuda else
                        ("native V5 runtime in host mode (CPU rehearsal: host engine, host transport over the "
                         "runtime's own TCP channel): " + ("root scatter every step -> overlap tiles -> gather"
                                                           if a.workload == "v4" else
                                                           "stage1 -> pool1 halo chunks -> stage2 -> gather"))
                        if not cuda else
                        ("device-resident input (placed once) -> " if a.input_source == "local" else
                         "root device -> scatter (every step) -> ") +
                        "stage1 (chunks) -> pool1 halo chunks -> stage2 (halo-free ranks: free-running lanes) -> "
                        "gather (native V5 runtime; gather on a second stream under the next step)")
            extra = {**wl.describe(), "workload": a.workload, "decomp": a.decomp, "phases_ms": phases}
            if a.workload == "v4" and cuda:
                gbps = wl.probe_h2d_gbps()
                per_img = extra["h2d_bytes_per_step_rank"] / max(1, -(-GB // world))
                extra.update({"h2d_gbps_link": round(gbps, 2),
                              "h2d_gbps_in_step": round(extra["h2d_bytes_per_step_rank"] / (phases["h2d"] * 1e6), 2)
                              if phases.get("h2d") else None,
                              "h2d_bound_img_s": round(world * gbps * 1e9 / per_img, 1),
                              "h2d_bound_fraction": round(imgs / (world * gbps * 1e9 / per_img), 3)})
            elif a.workload == "v4":
                extra["lanes"] = a.lanes
        # the modelled 1/2/4/8-GPU curve of this configuration (anx/cost.hpp; measured: false), with
        # this run's measured rate in the throughput table when it ran on one GPU
        model = None
        if cuda:
            from anx.parallel import cost
            wl_name = "dp" if wl is None else a.workload
            per_gpu = B if wl is None else GB
            ov = {}
            if world == 1 and wl_name in ("dp", "v5"):
                pts = dict(cost.curve(wl_name, per_gpu)["params"]["rate"])
                pts[B if wl is None else GB] = round(imgs)
                ov["rate"] = ",".join(f"{k}:{v}" for k, v in sorted(pts.items()))
            model = cost.curve(wl_name, per_gpu, input_source=a.input_source if wl_name != "v4" else "root",
                               mode="per_layer", overrides=ov)
            model.pop("steps", None)
        rec = {
            "metric": METRIC,
            "value": round(imgs, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": scaling,
            # like for like with the reference's headline (one image through a fresh process: context,
            # allocation, H2D + forward + D2H): 610.661 ms / our process-cold batch-1 time
            "vs_baseline": b1p.get("b1_process_cold_vs_reference"),
            "vs_baseline_kind": "cold single image, fresh process (reference V3 610.661 ms / b1_process_cold_ms)",
            "dtype": "fp32",
            "data": ("synthetic (U[0,0.1) images 227x227x3 generated on %s, random-init weights)"
                     % ("each rank" if wl is None and a.input_source == "local" else "rank 0")),
            "config": {
                "model": MODEL,
                "workload": a.workload,
                "global_batch": per_step,
                "seq_len": None,
                "image": [d.H, d.W, d.C0],
                "parallelism": par,
                "pipeline": pipeline,
                "impl": a.impl,
                **extra,
                "ms_per_batch": round(ms, 4),
                "prewarm_steps": n_pw,
                "prewarm_ms": prewarm_ms,
                "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                "gflop_per_image_direct": round(anx.flops_per_image() / 1e9, 4),
                "gflop_per_image_mfma": round(mf / 1e9, 4),
                "direct_equiv_tflops": round(imgs * anx.flops_per_image() / 1e12, 2),
                "mfma_tflops": round(imgs * mf / 1e12 / world, 2),
                "mfma_tflops_note": "per GPU; fp32 matrix peak 157 TF/s (155 sustained)",
                "vs_baseline_throughput": round(imgs / (1000.0 / BASELINE_V3_MS), 1),
                **b1p,
            },
        }
        if world > 1:  # who ran and whether the gathered outputs are right (selfcheck)
            rec["rccl_world_size"] = ident["world_size"] if ident else world
            rec["identity"] = ident
            if verify is not None:
                rec["gather_verified"] = verify["gather_verified"]
                rec["verify"] = verify
        if model is not None:  # modelled, not measured: outside the measured config
            rec["model_curve"] = {"measured": False, **model}

    # Secondary records, after the headline is measured and its record built. Their native multi-GPU
    # programs (V4 / V5 over RCCL and peer IPC) meet real multi-GPU hardware for the first time in the
    # driver's N > 1 runs: a hung call there must not take the headline line with it (SecondaryDeadline).
    t_sec = time.perf_counter()
    guard = selfcheck.SecondaryDeadline(rank, a.secondary_deadline_s, rec,
                                        hang=os.environ.get("ANX_BENCH_HANG_STAGE"))  # hang: tests only
    guard.stage("v5_subrecords")
    subs = {}
    if cuda and wl is not None and a.workload == "v5" and not a.no_subrecords:
        subs = v5_halo_subrecords(a, world, rank, GB, dev, g)
    guard.stage("batch1")
    b1 = batch1_latency(dev) if (rank == 0 and cuda and not a.no_b1) else {}
    guard.stage("reference_programs")
    refs = None
    if wl is None and a.model == "blocks" and not a.no_ref_programs:
        try:
            refs = reference_programs(a, world, rank, dev, cuda, g)
        except Exception as e:
            refs = {"error": repr(e)[:300]}
    guard.stage("full_bf16")
    full = None
    if cuda and wl is None and not a.no_full:
        try:
            full = full_bf16_secondary(dev, world, rank)
        except Exception as e:  # the headline record must not depend on the extension
            full = {"error": repr(e)[:300]}
    guard.stage("closing barrier")
    if rank == 0:
        rec["config"].update(b1)
        if full is not None:
            rec["full_bf16"] = full
        if refs is not None:
            rec.update(refs) if "error" not in refs else rec.update({"reference_programs_error": refs["error"]})
        rec.update(subs)
        rec["secondary_s"] = round(time.perf_counter() - t_sec, 1)
        guard.emit(rec)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    guard.done()


if __name__ == "__main__":
    main()
