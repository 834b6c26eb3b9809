"""Batch-parallel scatter -> compute -> gather pipeline over torch.distributed (RCCL on GPUs,
gloo on CPU ranks).

This is the reference's V4/V5 program shape — rank 0 owns the input, ``MPI_Scatterv`` rows out,
compute, ``MPI_Gatherv`` back (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:52-130) — at
batch scale and MI355X-first:

* the decomposition axis is the batch (images are independent; no halo traffic at all), the
  row/halo decomposition of single images lives in the native V4 / V5 runtimes
  (:mod:`anx.parallel.workloads`);
* collectives are RCCL scatter/gather (grouped point-to-point from/to the root, one direct xGMI
  link per peer) issued asynchronously on RCCL's stream, split into micro-batches so the scatter
  of micro-batch i+1 and the gather of i-1 overlap the compute of i on the compute stream;
* buffers are allocated once and reused every step (the reference re-mallocs per call, D5);
* ``prefetch=True`` pipelines ACROSS steps: the input of step k+1 is scattered into the second of
  two input buffers while step k computes, so the root's xGMI egress (world-1 links, each carrying
  one peer's shard) overlaps the compute instead of preceding it. Every step still scatters,
  computes and gathers its full batch; only the order changes.

* ``async_lanes=True`` (local input only): a model with stream lanes runs them free (its
  ``forward_async``: no per-step join, lanes half a forward apart) and each lane gathers its own
  slice from its own stream; a lane waits, on its stream, for the gather that read the same output
  buffer two steps earlier. ``drain()`` joins the lanes.

``root_batch`` (local input, dp): rank 0 computes only that many images per step while every peer
computes ``batch_per_rank`` -- the root also receives the whole gather, and that receive costs it
compute (11-18 % at the 8-GPU volume, tools/probe_ingest.py), so it sheds the share the cost model
prices (:func:`anx.parallel.cost.dp_root_batch`). The reference's root likewise gets its own
Scatterv count (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:52-75, counts per rank). Unequal
slices cannot use ``gather``, so each segment goes point to point: peers ``isend`` their segment,
the root ``irecv``s every peer's segment in one batch into ``y_global[r, seg]`` and copies its own
slice into ``y_global[0]`` (rows past ``root_batch`` of ``y_global[0]`` are unused).

``inputs`` (local input only): a list of input batches used round-robin, step k computing
``inputs[k % len(inputs)]`` (its first rows: this rank's share) — a benchmark streams distinct data
through the engine instead of one cache-resident batch. ``x_used`` is the batch the last step computed.

``set_root_batch(n)`` changes the root's share between steps (after :meth:`drain`; the root's buffers
are allocated for ``batch_per_rank`` rows and sliced), so a benchmark can calibrate it from measured
per-rank compute (``timing = True``: every async step records each lane's compute span — from the end
of its wait for the gather that last read its output slice to the end of its forward, before its own
gather — as HIP events, or host time on CPU ranks; :meth:`lane_span_ms` is the mean span per step).

Input semantics with prefetch: ``step()`` snapshots ``x_global`` as it is at the call (the scatter
for the NEXT step is issued from it) and computes the batch snapshotted by the previous call (the
first call computes its own snapshot). Writes to ``x_global`` after ``step()`` returns are safe when
they are stream-ordered on the current stream (any torch op or copy): each step makes the current
stream wait for the scatter it issued before returning, so a later write cannot overtake that read.
Host code writing ``x_global`` through a raw pointer must synchronise the stream first.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def micro_splits(B: int, M: int) -> list[tuple[int, int]]:
    M = max(1, min(M, B)) if B > 0 else 1
    sizes = [B // M + (1 if i < B % M else 0) for i in range(M)]
    out, lo = [], 0
    for s in sizes:
        out.append((lo, lo + s))
        lo += s
    return out


def root_batch_for(rb: int, batch: int, micro: int, lane_bounds=None) -> tuple[int, str | None]:
    """The root's share ``rb`` (e.g. the cost model's :func:`anx.parallel.cost.dp_root_batch`) made valid
    for :meth:`ScatterComputeGather.set_root_batch`: the root must split its share into as many
    micro-batches and stream lanes as a peer's ``batch`` (per-lane gathers pair lane i of every rank).
    ``lane_bounds(n)``: the model's lane split (``AlexNetBlocks.lane_bounds`` or :func:`split_lanes`).
    Returns the share (raised to the smallest valid one, never above ``batch``) and a note when it moved.
    round-4/5 ADVICE: 8 GPUs x 32 images shed the root to 30, one lane against its peers' two."""
    rb = max(1, min(int(rb), batch))
    need = min(max(1, micro), batch)  # micro_splits(rb, M) must have as many parts as micro_splits(B, M)
    if lane_bounds is not None:
        lanes_b = len(lane_bounds(batch)) - 1
        lo, hi = max(rb, need), batch
        while lo < hi and len(lane_bounds(lo)) - 1 != lanes_b:  # lane counts grow with n: smallest valid share
            lo += 1
        need = lo
    out = max(rb, need)
    note = None if out == rb else f"root share {rb} raised to {out}: the root runs as many lanes / micro-batches as a peer"
    return out, note


@dataclass
class PipelineConfig:
    batch_per_rank: int
    micro: int = 4
    scatter: bool = True   # rank 0 owns the global batch and scatters it
    gather: bool = True    # outputs are gathered to rank 0
    prefetch: bool = False  # scatter step k+1 while step k computes (double-buffered x and y)
    async_lanes: bool = False  # free-running model lanes (forward_async) with per-lane gathers; local input only
    root_batch: int | None = None  # images rank 0 computes per step (local input; None = batch_per_rank)


class ScatterComputeGather:
    """One step: ``x_global[world, B, ...]`` (rank 0) -> per-rank ``model`` -> ``y_global`` (rank 0).

    ``model(x, out=y)`` must run asynchronously on the current stream (AlexNetBlocks does).
    """

    def __init__(self, model, cfg: PipelineConfig, in_shape, out_shape, device, group=None):
        self.model, self.cfg, self.device, self.group = model, cfg, torch.device(device), group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        B = cfg.batch_per_rank
        M = cfg.micro if self.world > 1 else 1
        self._M = M
        self.peer_splits = micro_splits(B, M)  # a peer's micro-batches (the root receives these)
        self.root_batch, self.shed = B, False
        self.prefetch = cfg.prefetch and self.world > 1
        nbuf = 2 if self.prefetch else 1
        # full batch_per_rank rows on every rank: the root's share is a slice (set_root_batch)
        self._xfull = [torch.empty((B, *in_shape), device=self.device) for _ in range(nbuf)]
        self._yfull = [torch.empty((B, *out_shape), device=self.device) for _ in range(nbuf)]
        self._n = B  # images this rank computes per step
        self.set_root_batch(B if cfg.root_batch is None or self.world == 1 else cfg.root_batch, _init=True)
        self._k = 0
        self._scatter_pending = None          # works that fill the input of the next step
        self._gather_pending = [None] * nbuf  # works still reading y buffer i
        # single rank: no scatter/gather buffers at all (the V3 shape: compute on resident data)
        root = self.rank == 0 and self.world > 1
        self.x_global = torch.empty((self.world, B, *in_shape), device=self.device) if root and cfg.scatter else None
        self.y_global = (torch.empty((self.world, cfg.batch_per_rank, *out_shape), device=self.device)
                         if root and cfg.gather else None)
        self.async_lanes = cfg.async_lanes and not cfg.scatter and hasattr(model, "forward_async")
        if self.async_lanes and self.world > 1 and cfg.gather and nbuf < 2:  # a gather may still read y[k-1]
            self._yfull.append(torch.empty_like(self._yfull[0]))
            self._gather_pending.append(None)
        self._slice_bufs()
        self._lane_gathers = [dict() for _ in self._yb]  # per output buffer: lane -> gather work reading it
        self.inputs: list | None = None  # local input only: batches used round-robin (see module doc)
        self.x_used = None  # the input batch the last step computed
        self.timing = False  # record per-lane compute spans (lane_span_ms)
        self._spans: list = []

    def _slice_bufs(self) -> None:
        n = self._n
        self._xb = [t[:n] for t in self._xfull]
        self._yb = [t[:n] for t in self._yfull]
        self.x, self.y = self._xb[0], self._yb[0]

    def set_root_batch(self, rb: int, _init: bool = False) -> None:
        """Images rank 0 computes per step (local input, dp). Only between steps, after :meth:`drain`.
        Every rank may call it (peers only validate): the root's lanes must split ``rb`` images into as
        many lanes, and micro-batches, as a peer's ``batch_per_rank``."""
        B, M = self.cfg.batch_per_rank, self._M
        rb = B if self.world == 1 else int(rb)
        if rb != B and (self.cfg.scatter or not 0 < rb <= B):
            raise ValueError(f"root_batch {rb} needs local input and 0 < root_batch <= batch_per_rank {B}")
        if rb != B and min(M, rb) != min(M, B):
            raise ValueError(f"root_batch {rb} must give the root as many micro-batches ({M}) as its peers")
        if rb != B and hasattr(self.model, "lane_bounds") and \
                len(self.model.lane_bounds(rb)) != len(self.model.lane_bounds(B)):
            raise ValueError(f"root_batch {rb} runs {len(self.model.lane_bounds(rb)) - 1} lanes, a peer's batch "
                             f"{B} {len(self.model.lane_bounds(B)) - 1}")
        self.root_batch, self.shed = rb, rb != B
        self._n = rb if self.rank == 0 else B
        self.splits = micro_splits(self._n, M)
        if not _init:
            self._slice_bufs()

    def lane_span_ms(self, reset: bool = True) -> float:
        """Mean compute span per step of this rank's lanes (ms) over the steps recorded with ``timing``
        (async steps only; syncs the device first on GPUs)."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        per_step = {}
        for k, lane, a, b in self._spans:
            ms = a.elapsed_time(b) if hasattr(a, "elapsed_time") else (b - a) * 1e3
            per_step.setdefault(k, []).append(ms)
        if reset:
            self._spans = []
        if not per_step:
            return 0.0
        return sum(sum(v) / len(v) for v in per_step.values()) / len(per_step)

    def _gather(self, y, seg: int, lo: int, hi: int):
        """Collect micro-batch / lane segment ``seg`` (this rank's rows [lo, hi) of ``y``) at rank 0."""
        root = self.rank == 0
        if not self.shed:
            dst = [self.y_global[r, lo:hi] for r in range(self.world)] if root else None
            return dist.gather(y[lo:hi], dst, dst=0, group=self.group, async_op=True)
        if not root:
            ops = [dist.P2POp(dist.isend, y[lo:hi], dist.get_global_rank(self.group, 0) if self.group else 0,
                              self.group)]
        else:
            self.y_global[0, lo:hi].copy_(y[lo:hi])
            plo, phi = self._peer_seg[seg]
            ops = [dist.P2POp(dist.irecv, self.y_global[r, plo:phi],
                              dist.get_global_rank(self.group, r) if self.group else r, self.group)
                   for r in range(1, self.world)]
        return _Works(dist.batch_isend_irecv(ops))

    def _local_input(self, default):
        if self.inputs and not self.cfg.scatter:
            x = self.inputs[self._k % len(self.inputs)][:self._n]
        else:
            x = default
        self.x_used = x
        return x

    def _mark(self):
        if self.device.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time
        return time.perf_counter()

    def _scatter(self, x):
        root = self.rank == 0
        works = []
        for lo, hi in self.splits:
            src = [self.x_global[r, lo:hi] for r in range(self.world)] if root else None
            works.append(dist.scatter(x[lo:hi], src, src=0, group=self.group, async_op=True))
        return works

    def _step_prefetch(self) -> None:
        cur = self._k % 2
        x, y = self._local_input(self._xb[cur]), self._yb[cur]
        if self.cfg.scatter and self._scatter_pending is None:  # pipeline fill (first step only)
            self._scatter_pending = self._scatter(x)
        mine = self._scatter_pending or []
        # prefetch the next step's input into the other buffer. RCCL orders it after everything
        # already enqueued on this stream (the previous step's compute, the last reader of that buffer).
        self._scatter_pending = self._scatter(self._xb[cur ^ 1]) if self.cfg.scatter else None
        for w in mine:
            w.wait()
        if self._gather_pending[cur] is not None:  # y[cur] is still being gathered from 2 steps ago
            for w in self._gather_pending[cur]:
                w.wait()
        gw = []
        self._peer_seg = self.peer_splits
        for j, (lo, hi) in enumerate(self.splits):
            self.model(x[lo:hi], out=y[lo:hi])
            if self.cfg.gather:
                gw.append(self._gather(y, j, lo, hi))
        self._gather_pending[cur] = gw
        # Order the prefetch's read of x_global before anything the caller enqueues next (e.g. writing
        # the following batch into x_global). Enqueued after this step's compute, so it delays
        # nothing: step k+1's compute needs that scatter anyway.
        for w in self._scatter_pending or []:
            w.wait()
        self.x, self.y = x, y
        self._k += 1

    def _step_async(self) -> None:
        cur = self._k % len(self._yb)
        y, pend = self._yb[cur], self._lane_gathers[cur]
        gather = self.cfg.gather and self.world > 1

        marks = {}

        def pre_lane(i, lo, hi):  # on lane i's stream: the gather of this slice two steps ago is done
            w = pend.pop(i, None)
            if w is not None:
                w.wait()
            if self.timing:
                marks[i] = self._mark()

        def on_lane(i, lo, hi):  # on lane i's stream: gather its slice as soon as it is computed
            if self.timing:
                self._spans.append((self._k, i, marks.pop(i), self._mark()))
            if gather:
                pend[i] = self._gather(y, i, lo, hi)

        x = self._local_input(self.x)
        if self.shed:  # the root's lanes split fewer images: it receives the peers' lane slices
            lanes = _lane_bounds(self.model, self.root_batch)
            if lanes != len(peer := _lane_bounds(self.model, self.cfg.batch_per_rank, bounds=True)) - 1:
                raise ValueError(f"root_batch {self.root_batch} runs {lanes} lanes, a peer's batch {len(peer) - 1}")
            self._peer_seg = list(zip(peer[:-1], peer[1:]))
        self.model.forward_async(x, y, on_lane=on_lane, pre_lane=pre_lane)
        self.y = y
        self._k += 1

    def drain(self) -> None:
        """Wait for every outstanding prefetch/gather (the last step's outputs are then in y_global)."""
        if self.async_lanes:
            self.model.join()
            for pend in self._lane_gathers:
                for w in pend.values():
                    w.wait()
                pend.clear()
        for ws in [self._scatter_pending or []] + [g or [] for g in self._gather_pending]:
            for w in ws:
                w.wait()
        self._gather_pending = [None] * len(self._gather_pending)

    def step(self) -> None:
        if self.async_lanes:
            return self._step_async()
        if self.prefetch:
            return self._step_prefetch()
        if self.world == 1:
            if self.x_global is not None:
                self.x.copy_(self.x_global[0])
            self.model(self._local_input(self.x), out=self.y)
            if self.y_global is not None:
                self.y_global[0].copy_(self.y)
            self._k += 1
            return
        sw = self._scatter(self.x) if self.cfg.scatter else []
        gw = []
        x = self._local_input(self.x)
        self._peer_seg = self.peer_splits
        for i, (lo, hi) in enumerate(self.splits):
            if sw:
                sw[i].wait()
            self.model(x[lo:hi], out=self.y[lo:hi])
            if self.cfg.gather:
                gw.append(self._gather(self.y, i, lo, hi))
        for w in gw:
            w.wait()
        self._k += 1


class _Works:
    """The works of one batched point-to-point exchange, waited as one (a gather's work stand-in)."""

    def __init__(self, works):
        self.works = works or []

    def wait(self):
        for w in self.works:
            w.wait()


def _lane_bounds(model, n: int, bounds: bool = False):
    """How ``model.forward_async`` splits ``n`` images over its lanes: the lane count, or (bounds=True)
    the lane boundaries [0, ..., n]."""
    b = model.lane_bounds(n) if hasattr(model, "lane_bounds") else [0, n]
    return b if bounds else len(b) - 1
