"""The five staged versions of the reference, as runnable programs on MI355X.

  v1    serial CPU                      (final_project/v1_serial; call stack SURVEY §3.1)
  v2.1  CPU ranks, broadcast-all        (v2_mpi_only/2.1_broadcast_all)
  v2.2  CPU ranks, scatter + halo       (v2_mpi_only/2.2_scatter_halo)
  v3    single GPU                      (v3_cuda_only)
  v4    GPU ranks, host-staged scatter/halo/gather (v4_mpi_cuda)
  v5    GPU ranks, device-resident RCCL scatter / per-layer halo / gather (v5_cuda_aware_mpi —
        empty in the reference, planned at README.md:158-166)

Each run prints the reference's stdout contract lines so its log parsers still work,
plus one JSON record: version, np, batch, per-phase ms (cold = first call incl. setup, warm =
steady-state mean), images/s, output shape, first values and a checksum, and (with --check) the
max error vs the single-process reference.

Multi-rank versions read RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* from the environment (torchrun, or
``python -m anx launch``); CPU ranks use gloo, GPU ranks RCCL (``nccl``). A GPU rank binds
``LOCAL_RANK % device_count`` — the binding the reference documented but never called (D4).
"""
from __future__ import annotations

import json
import os
import time
import zlib
from dataclasses import asdict, dataclass, field

import torch
import torch.distributed as dist

from .config import blocks_dims, flops_per_image
from .parallel import comm
from .parallel.plan import OVERLAP, PER_LAYER
from .parallel.tensor import filter_parallel_forward
from .utils.init import init_input, init_weights
from .utils.timer import PhaseTimer

VERSIONS = ("v1", "v2.1", "v2.2", "v3", "v4", "v5")


@dataclass
class RunConfig:
    version: str = "v3"
    batch: int = 1
    init: str = "const"
    seed: int = 0
    lrn_mode: str | None = None   # default: div_n for v1/v2.x, raw for v3..v5 (reference parity, D1)
    groups2: int = 1
    decomp: str | None = None     # overlap | per_layer (default: overlap, per_layer for v5)
    strategy: str = "rows"        # rows | batch | filter (multi-rank versions)
    iters: int = 0                # warm iterations after the cold run
    impl: str = "mfma"
    check: bool = False
    quiet: bool = False
    cpu_rehearsal: bool = False   # run the GPU versions' program on CPU ranks over gloo (tests)
    conv2_algo: str = "auto"      # auto | direct | winograd (direct = bit-identical across decompositions)
    conv1_algo: str = "auto"      # auto | direct | winograd (likewise for Conv1's polyphase Winograd)


@dataclass
class RunResult:
    version: str
    np: int
    batch: int
    shape: list
    first10: list
    checksum: int
    cold_ms: float
    warm_ms: float | None
    images_per_s: float | None
    phases_cold: dict = field(default_factory=dict)
    phases_warm: dict = field(default_factory=dict)
    max_abs_err: float | None = None
    lrn_mode: str = ""
    decomp: str = ""
    strategy: str = ""
    device: str = ""
    tflops: float | None = None


def _defaults(cfg: RunConfig) -> RunConfig:
    if cfg.version not in VERSIONS:
        raise ValueError(f"version must be one of {VERSIONS}")
    if cfg.lrn_mode is None:
        cfg.lrn_mode = "div_n" if cfg.version in ("v1", "v2.1", "v2.2") else "raw"
    if cfg.decomp is None:
        cfg.decomp = PER_LAYER if cfg.version == "v5" else OVERLAP
    return cfg


def _init_dist(backend: str) -> tuple[int, int]:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dev = torch.device("cuda", torch.cuda.current_device())
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return comm.world()


def _checksum(y: torch.Tensor) -> int:
    return zlib.crc32(y.detach().float().cpu().contiguous().numpy().tobytes()) & 0xFFFFFFFF


def _native_runtime(cfg: RunConfig, w: dict | None, b1, b2, gpu: bool):
    """Multi-rank row / image splits run on the native runtimes (libanx_dist), CPU and GPU alike:
    V4 on GPUs = the host-staged runtime (anx/v4.hpp; a per_layer V4 runs V5's schedule with the
    batch on the root), V5 = the device-resident runtime (anx/v5.hpp), V2.2 and the CPU rehearsals = the
    V5 runtime in host mode (host engine + host transport). Every step starts from the root's batch,
    as the reference's programs did."""
    from .parallel.workloads import NativeV4, NativeV5
    decomp = "batch" if cfg.strategy == "batch" else "rows"
    if not gpu:
        return NativeV5(cfg.batch, w, specs=(b1, b2), decomp=decomp, layer=cfg.decomp, impl="host",
                        input_source="root")
    for k, v in (("ANX_CONV1_ALGO", cfg.conv1_algo), ("ANX_CONV2_ALGO", cfg.conv2_algo)):
        if v != "auto":  # knob seeds of the runtimes' engines
            os.environ[k] = v
    if cfg.version == "v4" and (cfg.decomp == OVERLAP or decomp == "batch"):
        return NativeV4(cfg.batch, w, specs=(b1, b2), decomp=decomp, impl=cfg.impl)
    return NativeV5(cfg.batch, w, specs=(b1, b2), decomp=decomp, layer=cfg.decomp, impl=cfg.impl,
                    input_source="root")


def run(cfg: RunConfig) -> RunResult | None:
    """Run one version; returns the result on rank 0 (None on other ranks)."""
    from .models.alexnet_blocks import AlexNetBlocks

    cfg = _defaults(cfg)
    gpu = cfg.version in ("v3", "v4", "v5") and not cfg.cpu_rehearsal
    if gpu:
        if not torch.cuda.is_available():
            raise RuntimeError(f"{cfg.version} needs a GPU")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % torch.cuda.device_count())
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    # the native runtimes carry their own transports; torch.distributed only broadcasts their port and
    # runs the Python strategies (broadcast-all, filter split)
    backend = "nccl" if (cfg.version == "v5" and gpu and cfg.strategy == "filter") else "gloo"
    t_start = time.perf_counter()
    rank, ws = _init_dist(backend)
    if cfg.version in ("v1", "v3") and ws > 1:
        raise RuntimeError(f"{cfg.version} is a single-process version (got WORLD_SIZE={ws})")
    comm_dev = device if cfg.version == "v5" else torch.device("cpu")  # v4 stages through the host

    timer = PhaseTimer(device, sync=True)
    from .config import blocks
    b1, b2 = blocks(cfg.lrn_mode, cfg.groups2)
    d = blocks_dims(b1=b1, b2=b2)
    native = model = None
    use_native = cfg.version in ("v2.2", "v4", "v5") and cfg.strategy in ("rows", "batch")
    with timer.phase("setup"):
        w = init_weights(cfg.init, cfg.seed, b1, b2) if rank == 0 else \
            {k: torch.empty_like(v) for k, v in init_weights("const", 0, b1, b2).items()}
        x = init_input(cfg.batch, cfg.init, cfg.seed) if rank == 0 else None
        if use_native:
            native = _native_runtime(cfg, w if rank == 0 else None, b1, b2, gpu)
            native.fill(x)
        else:
            w = comm.bcast_weights(w, device=comm_dev)
            model = AlexNetBlocks(w, specs=(b1, b2), device=device, impl=cfg.impl, max_batch=cfg.batch,
                                  knobs={"conv1_algo": cfg.conv1_algo, "conv2_algo": cfg.conv2_algo} if gpu else None)
        if cfg.version == "v2.1" or (cfg.strategy == "filter" and cfg.version in ("v2.2", "v4", "v5")):
            # broadcast-all: every rank receives the whole input (M3, main.cpp:71); the filter
            # (tensor-parallel) strategy also replicates Block 1 and needs the whole input
            xb = x if rank == 0 else torch.empty(cfg.batch, d.H, d.W, d.C0)
            if ws > 1:
                xb = xb.to(device) if backend == "nccl" else xb  # RCCL broadcasts device memory
                dist.broadcast(xb, 0)
            x = xb
        if x is not None and native is None:
            x = x.to(comm_dev if cfg.version in ("v4", "v5") else device)

    def once(tm: PhaseTimer):
        if cfg.version in ("v1", "v3", "v2.1"):
            xx = x
            if cfg.version == "v3" and device.type == "cuda":
                with tm.phase("h2d"):
                    xx = x.to(device)
            # P1 "broadcast-all" (V2.1, v2_mpi_only/2.1_broadcast_all/src/main.cpp:49-85) and V1 / V3: every
            # rank computes the whole batch, rank 0's result is the answer (no gather, as the reference)
            with tm.phase("compute"):
                y = model(xx)
            if cfg.version == "v3" and device.type == "cuda":
                with tm.phase("d2h"):
                    y = y.cpu()
            return y if rank == 0 else None
        if native is not None:
            with tm.phase("step"):
                native.step()
                native.sync()
            return native.output()
        if cfg.strategy == "filter":
            with tm.phase("compute"):
                return filter_parallel_forward(x.to(device), model.weights, b1, b2, gather="root",
                                               comm_device=comm_dev)
        raise ValueError(f"{cfg.version} with strategy {cfg.strategy!r} at np={ws}")

    if ws > 1:
        dist.barrier()
    with timer.phase("total"):
        y = once(timer)
    phases_cold = dict(timer.ms)
    if native is not None:  # the runtime's own per-phase split of the step
        phases_cold.update({f"step.{k}": v for k, v in native.phase_ms(reset=True).items()})
    cold_ms = phases_cold.pop("total") + phases_cold.get("setup", 0.0)
    phases_cold["wall_since_start"] = (time.perf_counter() - t_start) * 1e3

    warm_ms = None
    phases_warm = {}
    if cfg.iters > 0:
        wt = PhaseTimer(device, sync=True)
        if ws > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(cfg.iters):
            y = once(wt)
        if device.type == "cuda":
            torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        warm_ms = (time.perf_counter() - t0) * 1e3 / cfg.iters
        phases_warm = wt.scaled(1.0 / cfg.iters)
        if native is not None:
            phases_warm.update({f"step.{k}": v for k, v in native.phase_ms().items()})

    res = None
    if rank == 0:
        y = y.float().cpu()
        err = None
        if cfg.check:
            from .models.reference import blocks_forward
            ref = blocks_forward(init_input(cfg.batch, cfg.init, cfg.seed), w if native else model.weights, b1, b2)
            err = float((y.double() - ref).abs().max())
        ips = cfg.batch / (warm_ms / 1e3) if warm_ms else None
        res = RunResult(cfg.version, ws, cfg.batch, list(y.shape[1:]), [round(float(v), 4) for v in y.flatten()[:10]],
                        _checksum(y), round(cold_ms, 3), None if warm_ms is None else round(warm_ms, 4),
                        None if ips is None else round(ips, 2), {k: round(v, 4) for k, v in phases_cold.items()},
                        {k: round(v, 4) for k, v in phases_warm.items()}, err, cfg.lrn_mode, cfg.decomp,
                        cfg.strategy, str(device),
                        None if ips is None else round(ips * flops_per_image(b1=b1, b2=b2) / 1e12, 3))
        if not cfg.quiet:
            print_contract(res)
    if native is not None:
        native.close()
    if ws > 1:
        dist.barrier()
    return res


def print_contract(r: RunResult) -> None:
    """The reference's stdout lines followed by one JSON line."""
    shape = "x".join(str(s) for s in r.shape)
    vals = " ".join(f"{v:g}" for v in r.first10)
    t = r.warm_ms if r.warm_ms is not None else r.cold_ms
    if r.version == "v1":
        d = blocks_dims()
        for name, (h, w_, c) in (("Input", (d.H, d.W, d.C0)), ("Conv1", (d.H1, d.W1, d.C1)),
                                 ("Pool1", (d.Hp1, d.Wp1, d.C1)), ("Conv2", (d.H2, d.W2, d.C2)),
                                 ("Pool2", (d.Hp2, d.Wp2, d.C2)), ("LRN2", (d.Hp2, d.Wp2, d.C2))):
            print(f"  [{name}] Dimensions: H={h}, W={w_}, C={c}")
        print(f"AlexNet Serial Forward Pass completed in {t:.3f} ms")
        print(f"Final Output (first 10 values): {vals}")
    elif r.version in ("v2.1", "v2.2"):
        print(f"shape: {shape}")
        print("Sample values: " + " ".join(f"{v:g}" for v in r.first10[:5]))
        print(f"Execution Time: {t:.3f} ms")
    elif r.version == "v3":
        print(f"AlexNet HIP Forward Pass completed in {t:.3f} ms")
        print(f"Final Output (first 10 values): {vals}")
    else:
        print(f"Final Output Shape: {shape}")
        print(f"Final Output (first 10 values): {vals}")
        print(f"AlexNet {'RCCL' if r.version == 'v5' else 'MPI'}+HIP Forward Pass completed in {t:.3f} ms")
    print("ANX_JSON " + json.dumps(asdict(r)), flush=True)
