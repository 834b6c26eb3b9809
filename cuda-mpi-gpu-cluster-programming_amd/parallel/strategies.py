"""Distributed forward strategies for AlexNet Blocks 1-2.

  * :func:`replicate_forward`  — P1 "broadcast-all" (V2.1, v2_mpi_only/2.1_broadcast_all/src/main.cpp:49-85):
    every rank computes the whole batch; rank 0's result is the answer (no gather, as the reference).
  * :func:`rows_forward`       — P2 spatial row decomposition (V2.2 CPU, V4 host-staged GPU, V5
    device-resident GPU): Scatterv of owned input rows, input-halo exchange, local tile compute,
    [V5: pool1-halo exchange between conv1 and conv2], Gatherv of output rows. Rows come from the
    exact planner, so every np gives the single-device result (the reference's did not, D2/D3).
  * :func:`batch_forward`      — P6 batch data parallelism (absent in the reference): scatter images,
    compute, gather — the pipelined form is :class:`anx.parallel.pipeline.ScatterComputeGather`.

Staging: ``comm_device='cpu'`` runs collectives on host tensors (gloo; V2.2 and the V4 host-staged
path with explicit H2D/D2H phases); ``comm_device=model.device`` keeps every byte on the GPU and
runs RCCL over xGMI (V5).
"""
from __future__ import annotations

import torch

from . import comm
from .plan import OVERLAP, PER_LAYER, Rows, make_plan
from ..utils.timer import PhaseTimer


def replicate_forward(model, x: torch.Tensor, timer: PhaseTimer | None = None):
    timer = timer or PhaseTimer(model.device, sync=False)
    with timer.phase("compute"):
        y = model(x)
    return y


def _own_rows_tensor(x_full, plan, rank, N, W, C, device, timer):
    """Scatterv the disjoint owned input rows, then exchange input halos so this rank holds
    exactly rows tile.inp (the reference's M9 + M10/M12)."""
    tile = plan.tiles[rank]
    with timer.phase("scatter"):
        own = comm.scatter_rows(x_full, plan.owned_in, (N, W, C), device)
    buf = torch.empty((N, tile.inp.size, W, C), device=device)
    if not tile.out.empty:
        o = plan.owned_in[rank]
        lo = max(o.lo, tile.inp.lo)
        hi = min(o.hi, tile.inp.hi)
        if hi > lo:
            buf[:, lo - tile.inp.lo:hi - tile.inp.lo].copy_(own[:, lo - o.lo:hi - o.lo])
    with timer.phase("halo_in"):
        comm.exchange(
            plan.in_halos,
            get=lambda r: own[:, r.lo - plan.owned_in[rank].lo:r.hi - plan.owned_in[rank].lo],
            put=lambda r, b: buf[:, r.lo - tile.inp.lo:r.hi - tile.inp.lo].copy_(b),
            recv_shape=lambda r: (N, r.size, W, C),
            device=device,
        )
    return buf


def rows_forward(model, x_full: torch.Tensor | None, N: int, *, decomp: str = OVERLAP, comm_device=None,
                 timer: PhaseTimer | None = None):
    """Row-decomposed forward of N images. ``x_full`` ([N,H,W,C], on ``comm_device``) is only read
    on rank 0. Returns the full [N,Hp2,Wp2,C2] output on rank 0 (on ``comm_device``), None elsewhere."""
    rank, ws = comm.world()
    dev = model.device
    cdev = torch.device(comm_device) if comm_device is not None else dev
    timer = timer or PhaseTimer(dev, sync=False)
    d = model.dims
    plan = make_plan(model.H, model.W, ws, decomp, model.b1, model.b2)
    tile = plan.tiles[rank]
    xt = _own_rows_tensor(x_full, plan, rank, N, model.W, d.C0, cdev, timer)
    if cdev != dev:
        with timer.phase("h2d"):
            xt = xt.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else xt.to(dev)
    if decomp == OVERLAP:
        with timer.phase("compute"):
            y = model.tile_forward(xt, tile) if not tile.out.empty else \
                torch.empty(model.out_shape(N, 0), device=dev)
    elif decomp == PER_LAYER:
        with timer.phase("compute"):
            if not tile.out.empty:
                model.stage1(xt, tile)
        wshape = lambda r: model.window_rows_shape(N, r.size)  # noqa: E731
        with timer.phase("halo_p1"):
            if cdev == dev:  # device-resident: window rows go straight into RCCL buffers
                comm.exchange(plan.p1_halos, get=lambda r: model.window_get(tile, r.lo, r.hi, N),
                              put=lambda r, b: model.window_put(tile, r.lo, b), recv_shape=wshape, device=dev)
            else:  # host-staged halo (V4's unused per-layer fn, alexnet_mpi_cuda.cu:113-136)
                comm.exchange(plan.p1_halos, get=lambda r: model.window_get(tile, r.lo, r.hi, N).cpu(),
                              put=lambda r, b: model.window_put(tile, r.lo, b.to(dev)), recv_shape=wshape,
                              device=cdev)
        with timer.phase("compute"):
            y = model.stage2(N, tile) if not tile.out.empty else torch.empty(model.out_shape(N, 0), device=dev)
    else:
        raise ValueError(decomp)
    if cdev != dev:
        with timer.phase("d2h"):
            y = y.to(cdev)
    with timer.phase("gather"):
        out = comm.gather_rows(y, [t.out for t in plan.tiles])
    return out


def batch_forward(model, x_full: torch.Tensor | None, N: int, *, comm_device=None, timer: PhaseTimer | None = None):
    """Images split over ranks (first N % np ranks get one more), computed whole, gathered to rank 0."""
    rank, ws = comm.world()
    dev = model.device
    cdev = torch.device(comm_device) if comm_device is not None else dev
    timer = timer or PhaseTimer(dev, sync=False)
    d = model.dims
    from .plan import split_rows
    parts = split_rows(N, ws)
    with timer.phase("scatter"):
        # images are rows of dim 0: reuse the row scatter on a [1, N, ...] view
        xv = x_full.unsqueeze(0) if x_full is not None else None
        mine = comm.scatter_rows(xv, parts, (1, model.H, model.W, d.C0), cdev)[0]
    if cdev != dev:
        with timer.phase("h2d"):
            mine = mine.to(dev)
    with timer.phase("compute"):
        y = model(mine.contiguous()) if parts[rank].size else torch.empty(model.out_shape(0), device=dev)
    if cdev != dev:
        with timer.phase("d2h"):
            y = y.to(cdev)
    with timer.phase("gather"):
        out = comm.gather_rows(y.unsqueeze(0), parts)
    return None if out is None else out[0]


__all__ = ["replicate_forward", "rows_forward", "batch_forward", "Rows"]
