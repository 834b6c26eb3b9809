"""The reference's multi-GPU programs as steady-state, strong-scaling benchmark steps
(``bench.py --workload v4|v5``), over torch.distributed (RCCL over xGMI).

The reference's V4 (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:52-130) keeps the batch on rank
0's host, scatters input rows, runs the tile forward and gathers output rows back to the host; its
planned V5 (README.md:157-166) keeps every byte on the device and exchanges per-layer halos between
GPUs. Here both are one class, a fixed global batch split by the hybrid planner
(:func:`anx.parallel.plan.make_hybrid_plan`: ``rows`` = the reference's pure row split over all ranks,
``hybrid`` = batch first, rows only below one image per rank, ``batch`` = images only):

    v4  root pinned host --H2D--> root GPU --RCCL scatter (images x input rows incl. halo)--> ranks
        --tile_forward (overlap tiles: no mid-network exchange)--> RCCL gather --D2H--> root pinned host
    v5  root GPU --RCCL scatter--> ranks --stage1 (conv1+pool1)--> RCCL pool1-halo exchange inside each
        row group (per_layer tiles) --stage2 (conv2+pool2+LRN)--> RCCL gather --> root GPU

Every transfer is a grouped point-to-point op (RCCL has no Scatterv/Gatherv; root-centred grouped
P2P drives one xGMI link per peer at once). Buffers are allocated once. Each phase ends
with a CUDA event on the compute stream (no host sync inside a step), so the per-phase times come
from event pairs after the timed loop.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .comm import world
from .plan import OVERLAP, PER_LAYER, HybridPlan, make_hybrid_plan

DECOMPS = {"rows": None, "hybrid": 0, "batch": 1}  # row_ways (None = all ranks)
PHASES = ("h2d", "scatter", "stage1", "halo_p1", "compute", "gather", "d2h")


def _p2p(ops):
    if not ops:
        return []
    return dist.batch_isend_irecv(ops)


class RowsWorkload:
    def __init__(self, model, batch: int, version: str = "v5", decomp: str = "rows", layer: str | None = None,
                 device=None):
        if version not in ("v4", "v5"):
            raise ValueError("version must be v4 or v5")
        self.model, self.version = model, version
        self.device = torch.device(device) if device is not None else model.device
        self.rank, self.world = world()
        self.layer = layer or (OVERLAP if version == "v4" else PER_LAYER)
        if version == "v4" and self.layer != OVERLAP:
            raise ValueError("v4 runs overlap tiles (host-staged, no mid-network exchange)")
        rw = DECOMPS[decomp]
        self.plan: HybridPlan = make_hybrid_plan(model.H, model.W, self.world, batch,
                                                 self.world if rw is None else rw, self.layer, model.b1, model.b2)
        d = model.dims
        self.in_shape, self.out_shape = (model.H, model.W, d.C0), (d.Hp2, d.Wp2, d.C2)
        p, r = self.plan, self.rank
        self.tile, self.im = p.tile(r), p.images_of(r)
        self.n = self.im.size if not self.tile.out.empty else 0
        dev = self.device
        t = self.tile
        self.root = r == 0
        # whole-image tiles (a row group of one rank) need no stage1/halo/stage2 split: the plain
        # forward (stream lanes, fused path) computes them
        self.whole = t.inp.size == model.H and t.out.size == d.Hp2
        if self.root:
            self.x_dev = torch.empty((batch, *self.in_shape), device=dev)
            self.y_dev = torch.empty((batch, *self.out_shape), device=dev)
        if self.root and self.whole:  # the root computes its images in place: no local copies
            self.x_loc, self.y_loc = self.x_dev[self.im.lo:self.im.lo + self.n], self.y_dev[self.im.lo:self.im.lo + self.n]
        else:
            self.x_loc = torch.empty((self.n, t.inp.size, model.W, d.C0), device=dev)
            self.y_loc = torch.empty((self.n, t.out.size, d.Wp2, d.C2), device=dev)
        if self.root:
            pin = dev.type == "cuda"
            self.x_host = torch.empty((batch, *self.in_shape), pin_memory=pin) if version == "v4" else None
            self.y_host = torch.empty((batch, *self.out_shape), pin_memory=pin) if version == "v4" else None
            # per-peer contiguous staging for row-sliced transfers (whole-image transfers go in place)
            self.x_stage, self.y_stage = {}, {}
            for q in range(1, self.world):
                tq, iq = p.tile(q), p.images_of(q)
                if tq.out.empty or iq.empty:
                    continue
                if tq.inp.size != model.H:
                    self.x_stage[q] = torch.empty((iq.size, tq.inp.size, model.W, d.C0), device=dev)
                if tq.out.size != d.Hp2:
                    self.y_stage[q] = torch.empty((iq.size, tq.out.size, d.Wp2, d.C2), device=dev)
        # pool1 halos of this rank's row group (global rank ids)
        g = p.group_of[r]
        base = sum(p.group_size[:g])
        self.halos = [(x.src + base, x.dst + base, x.rows) for x in p.row_plans[g].p1_halos] \
            if self.layer == PER_LAYER else []
        self.halo_recv = {}
        for src, dst, rows in self.halos:
            if dst == r and self.n:
                self.halo_recv[(src, rows.lo)] = torch.empty(model.window_rows_shape(self.n, rows.size), device=dev)
        self._events = []

    # ------------------------------------------------------------------ data
    def fill(self, x: torch.Tensor) -> None:
        """Root only: the global batch [B,H,W,C] (host pinned for v4, device for v5)."""
        if self.root:
            (self.x_host if self.version == "v4" else self.x_dev).copy_(x)

    def output(self) -> torch.Tensor | None:
        """Root: the gathered output of the last step (host for v4, device for v5)."""
        if not self.root:
            return None
        return self.y_host if self.version == "v4" else self.y_dev

    # ------------------------------------------------------------------ one step
    def _mark(self, rec):
        if rec is not None and self.device.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            rec.append(e)

    def step(self, record: bool = False) -> None:
        p, r, m, t = self.plan, self.rank, self.model, self.tile
        rec = [] if record else None
        self._mark(rec)
        # h2d (v4): the root's batch from pinned host memory
        if self.root and self.version == "v4":
            self.x_dev.copy_(self.x_host, non_blocking=True)
        self._mark(rec)
        # scatter: each rank its images x input rows (tile.inp includes the overlap halo)
        ops = []
        if self.root:
            for q in range(self.world):
                tq, iq = p.tile(q), p.images_of(q)
                if tq.out.empty or iq.empty:
                    continue
                src = self.x_dev[iq.lo:iq.hi, tq.inp.lo:tq.inp.hi]
                if q == 0:
                    if not self.whole:
                        self.x_loc.copy_(src)
                    continue
                buf = self.x_stage.get(q)
                if buf is not None:
                    buf.copy_(src)
                else:
                    buf = self.x_dev[iq.lo:iq.hi]
                ops.append(dist.P2POp(dist.isend, buf, q))
        elif self.n:
            ops.append(dist.P2POp(dist.irecv, self.x_loc, 0))
        for w in _p2p(ops):
            w.wait()
        self._mark(rec)
        if self.layer == PER_LAYER and not self.whole:
            if self.n:
                m.stage1(self.x_loc, t)
            self._mark(rec)
            ops, sends = [], []
            for src, dst, rows in self.halos:
                if src == r and self.n:
                    b = m.window_get(t, rows.lo, rows.hi, self.n)
                    sends.append(b)
                    ops.append(dist.P2POp(dist.isend, b, dst))
                elif dst == r and self.n:
                    ops.append(dist.P2POp(dist.irecv, self.halo_recv[(src, rows.lo)], src))
            for w in _p2p(ops):
                w.wait()
            for src, dst, rows in self.halos:
                if dst == r and self.n:
                    m.window_put(t, rows.lo, self.halo_recv[(src, rows.lo)])
            self._mark(rec)
            if self.n:
                m.stage2(self.n, t, out=self.y_loc)
        else:
            self._mark(rec)
            self._mark(rec)
            if self.n:
                if t.inp.size == m.H:
                    m(self.x_loc, out=self.y_loc)  # whole images: the lane-split forward
                else:
                    m.tile_forward(self.x_loc, t, out=self.y_loc)
        self._mark(rec)
        # gather output rows to the root
        ops, recvs = [], []
        if self.root:
            for q in range(self.world):
                tq, iq = p.tile(q), p.images_of(q)
                if tq.out.empty or iq.empty:
                    continue
                dst = self.y_dev[iq.lo:iq.hi, tq.out.lo:tq.out.hi]
                if q == 0:
                    if not self.whole:
                        dst.copy_(self.y_loc)
                    continue
                buf = self.y_stage.get(q)
                if buf is None:
                    buf = self.y_dev[iq.lo:iq.hi]
                else:
                    recvs.append((dst, buf))
                ops.append(dist.P2POp(dist.irecv, buf, q))
        elif self.n:
            ops.append(dist.P2POp(dist.isend, self.y_loc, 0))
        for w in _p2p(ops):
            w.wait()
        for dst, buf in recvs:
            dst.copy_(buf)
        self._mark(rec)
        if self.root and self.version == "v4":
            self.y_host.copy_(self.y_dev, non_blocking=True)
        self._mark(rec)
        if rec is not None:
            self._events.append(rec)

    def phase_ms(self) -> dict:
        """Mean per-phase ms over the recorded steps (call after a device synchronize)."""
        if not self._events:
            return {}
        tot = {k: 0.0 for k in PHASES}
        for ev in self._events:
            for k, a, b in zip(PHASES, ev[:-1], ev[1:]):
                tot[k] += a.elapsed_time(b)
        n = len(self._events)
        return {k: round(v / n, 4) for k, v in tot.items()
                if v > 0 or k in ("scatter", "compute", "gather")}

    def describe(self) -> dict:
        p = self.plan
        return {"workload": self.version, "layer": self.layer, "groups": p.groups,
                "ranks_per_group": sorted(set(p.group_size)),
                "images_per_rank_max": max(p.images_of(q).size for q in range(self.world))}
