"""AlexNet Blocks 1-2 model (Conv1 11x11/4 -> ReLU -> MaxPool 3/2 -> Conv2 5x5/1 p2 -> ReLU ->
MaxPool 3/2 -> LRN 5), NHWC float32, backed by the native engine.

Parity with the reference's forward entry points:
  * V1 ``alexnetForwardPass``            final_project/v1_serial/src/alexnet_serial.cpp:67-186
  * V3 ``alexnetForwardPassCUDA``        final_project/v3_cuda_only/src/alexnet_cuda.cu:22-95
  * V4 ``alexnetTileForwardCUDA``        final_project/v4_mpi_cuda/src/alexnet_mpi_cuda.cu:157-205
    -> :meth:`AlexNetBlocks.tile_forward` (device tile of arbitrary height, exact row plan)
  * V4's unused per-layer ``alexnetForwardPassMPI_CUDA`` (:40-154)
    -> :meth:`stage1` / :meth:`window_get` / :meth:`window_put` / :meth:`stage2`
       (per-layer halo exchange, the V5 path)

On a GPU every call runs the libanx HIP kernels on torch's current stream (no host sync, graph
capturable). With ``lanes=L > 1`` a full-image forward of at least ``L * LANE_MIN`` images is split
into L contiguous slices, each run by its own engine (own workspace, same weights) on its own HIP
stream forked from and joined back to the current stream: the HBM-bound transforms and pools of one
lane fill the CUs the MFMA GEMMs of the other leave idle in their tail waves
(``profiles/r01_streams_probe.jsonl``: 2 x 150 images 1.362 ms vs 1 x 300 1.408 ms). Per-image
results are bit-identical to one lane. :meth:`forward_async` is the throughput form for repeated
forwards: the lanes are not joined per call but run free on their own streams, started half a
forward apart, so one lane's HBM-bound kernels overlap the other's GEMMs in steady state
(``profiles/r02_lanes_async.txt``: 128 images 0.629 -> 0.561 ms per forward). On the CPU it runs libanx's C++ host engine (CpuBlocks). There is no eager-PyTorch
fallback: the PyTorch oracle lives in :mod:`anx.models.reference` and is only used by tests.
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native as nat
from ..config import IN_H, IN_W, BlockSpec, blocks, blocks_dims
from ..parallel.plan import TilePlan, full_plan
from ..utils.init import init_weights
from ..utils.tuning import apply_knobs, knob_value, read_knob

IMPLS = {"mfma": 0, "direct": 1}
LANE_MIN = 16  # images per lane below which a forward stays on one stream (Winograd needs > 8)


def split_lanes(n: int, lanes: int) -> list[int]:
    """Image boundaries [0, ..., n] of ``n`` images over ``lanes`` stream lanes: one lane below
    ``lanes * LANE_MIN`` images, else contiguous near-equal slices (pure arithmetic: the CPU tests check
    the multi-GPU root share against it without a GPU)."""
    if lanes <= 1 or n < lanes * LANE_MIN:
        return [0, n]
    return [n * i // lanes for i in range(lanes + 1)]


def _tile_c(t: TilePlan) -> nat.TileC:
    return nat.TileC(t.inp.lo, t.inp.hi, t.c1.lo, t.c1.hi, t.p1.lo, t.p1.hi, t.q.lo, t.q.hi, t.c2.lo, t.c2.hi,
                     t.out.lo, t.out.hi)


def _check_hw_queues(lanes: int) -> None:
    """HIP maps a process's streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by default on
    MI355X): two lanes on one queue serialise (0.80 vs 0.57 ms per 128-image step,
    profiles/r02_lanes_async.txt). A lane model uses lanes + 1 streams (the caller's and its own)."""
    import os
    import warnings
    q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    if q < lanes + 1:
        warnings.warn(f"AlexNetBlocks(lanes={lanes}) uses {lanes + 1} streams but GPU_MAX_HW_QUEUES={q}: lanes "
                      "sharing a hardware queue serialise (set GPU_MAX_HW_QUEUES >= 8 before the first GPU call, "
                      "as bench.py does)", RuntimeWarning, stacklevel=3)


class AlexNetBlocks:
    def __init__(self, weights: dict | None = None, *, init: str = "const", seed: int = 0, lrn_mode: str = "div_n",
                 groups2: int = 1, H: int = IN_H, W: int = IN_W, device="cuda", impl: str = "mfma",
                 max_batch: int = 1, specs: tuple[BlockSpec, BlockSpec] | None = None, lanes: int = 1,
                 knobs: dict | None = None, lane_priority: int = 0):
        self.b1, self.b2 = specs if specs is not None else blocks(lrn_mode, groups2)
        if self.b1.has_lrn:
            raise ValueError("the native engine implements LRN after block 2 only (the reference's topology)")
        if self.b1.conv.P != 0:
            raise ValueError("conv1 padding must be 0 (row tiles read raw image rows)")
        self.H, self.W = H, W
        self.dims = blocks_dims(H, W, self.b1, self.b2)
        src = weights if weights is not None else init_weights(init, seed, self.b1, self.b2)
        self.weights = {k: v.detach().to("cpu", torch.float32).contiguous() for k, v in src.items()}
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if impl not in IMPLS:
            raise ValueError(f"impl must be one of {sorted(IMPLS)}")
        self.impl = impl
        # kernel knobs of this model's engines (anx.utils.tuning): applied at every engine creation
        self.knobs = {k: knob_value(k, v) for k, v in (knobs or {}).items()}
        self._engine = None
        self._cap = 0
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        multi = lanes > 1 and self.is_cuda
        per_lane = -(-max(1, max_batch) // lanes)
        # lane 0's engine runs slice 0, or the whole batch when it is too small to split
        self._ensure(max(per_lane, min(max_batch, lanes * LANE_MIN - 1)) if multi else max_batch)
        # side lanes (GPU only): engines for slices 1..L-1, each on its own stream; slice 0 runs here
        self._lanes: list[AlexNetBlocks] = []
        self._lane_streams: list[torch.cuda.Stream] = []
        if multi:
            _check_hw_queues(lanes)
            for _ in range(lanes - 1):
                self._lanes.append(AlexNetBlocks(self.weights, specs=(self.b1, self.b2), H=H, W=W, device=self.device,
                                                 impl=impl, max_batch=per_lane, knobs=self.knobs))
                # lane_priority < 0: side lanes on high-priority streams (their waves dispatch first)
                self._lane_streams.append(torch.cuda.Stream(self.device, priority=lane_priority))
        self._own_stream = None  # lane 0's stream in forward_async (the joined forward uses the current one)
        # forward_async from idle lanes: all lanes start together (False, default) or lane i after lane
        # i-1's stage 1, half a forward apart (True). With the fused transforms the staggered start no
        # longer pays in steady state (257.2 / 256.0 k vs 258.3 / 257.5 k images/s over 200 steps) and
        # its pipeline fill costs a short timed window ~1.5 % (20 steps: 250.5 / 249.6 k vs 253.0 /
        # 254.4 k; profiles/r03_stagger_bench_ab.jsonl)
        self.stagger = False

    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"

    def set_knob(self, name: str, value) -> None:
        """Change one kernel knob of this model (every lane); later forwards use it."""
        v = knob_value(name, value)
        if self.is_cuda and self._engine is not None:
            apply_knobs(self._engine, {name: v})
        self.knobs[name] = v
        for m in self._lanes:
            m.set_knob(name, v)

    def get_knob(self, name: str) -> int:
        """The value the GPU engine launches with."""
        if not self.is_cuda:
            raise ValueError("kernel knobs belong to the GPU engine")
        return read_knob(self._engine, name)

    # ------------------------------------------------------------------ engine lifetime
    def _ensure(self, n: int) -> None:
        if self._engine is not None and (n <= self._cap or not self.is_cuda):
            return
        self._close_engine()  # this engine only: the side lanes keep theirs
        h = C.c_void_p()
        w = self.weights
        args = (C.byref(nat.block_c(self.b1)), C.byref(nat.block_c(self.b2)), self.H, self.W, w["w1"].data_ptr(),
                w["b1"].data_ptr(), w["w2"].data_ptr(), w["b2"].data_ptr())
        if self.is_cuda:
            with torch.cuda.device(self.device):
                nat.call("anx_engine_create", C.byref(h), *args, max(1, n), IMPLS[self.impl])
            try:
                apply_knobs(h, self.knobs)
            except Exception:
                nat.lib().anx_engine_destroy(h)
                raise
        else:
            nat.call("anx_cpu_engine_create", C.byref(h), *args)
        self._engine, self._cap = h, max(1, n)

    def close(self) -> None:
        for m in getattr(self, "_lanes", ()):
            m.close()
        self._close_engine()

    def _close_engine(self) -> None:
        if self._engine is not None:
            if self.is_cuda:
                torch.cuda.synchronize(self.device)
                nat.lib().anx_engine_destroy(self._engine)
            else:
                nat.lib().anx_cpu_engine_destroy(self._engine)
            self._engine = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ shapes
    def out_shape(self, N: int, rows: int | None = None) -> tuple[int, int, int, int]:
        d = self.dims
        return (N, d.Hp2 if rows is None else rows, d.Wp2, d.C2)

    def _check_in(self, x: torch.Tensor, rows: int) -> int:
        if x.dim() != 4 or tuple(x.shape[1:]) != (rows, self.W, self.dims.C0):
            raise ValueError(f"expected NHWC input [N,{rows},{self.W},{self.dims.C0}], got {tuple(x.shape)}")
        if x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError("input must be contiguous float32")
        if x.device != self.device:
            raise ValueError(f"input on {x.device}, model on {self.device}")
        return x.shape[0]

    def _out(self, out: torch.Tensor | None, N: int, rows: int | None = None) -> torch.Tensor:
        """``out`` checked against the output the kernels will write (shape, dtype, layout, device), or a
        new tensor: the native engines write through the raw pointer."""
        shape = self.out_shape(N, rows)
        if out is None:
            return torch.empty(shape, device=self.device)
        if tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous() or out.device != self.device:
            raise ValueError(f"out must be a contiguous float32 {shape} tensor on {self.device}, got "
                             f"{tuple(out.shape)} {out.dtype} on {out.device}")
        return out

    def _stream(self) -> int:
        return nat.stream_ptr(self.device)

    # ------------------------------------------------------------------ forward paths
    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Full images: [N,H,W,3] -> [N,Hp2,Wp2,K2]."""
        plan = full_plan(self.H, self.W, self.b1, self.b2)
        if plan.inp.size != self.H and x.dim() == 4 and x.shape[1] == self.H:
            # a spec whose receptive field skips the last input rows (e.g. a 2x2 pool1): the tile reads
            # exactly the rows it needs
            x = x[:, plan.inp.lo:plan.inp.hi].contiguous()
        L = 1 + len(self._lanes)
        N = x.shape[0] if x.dim() == 4 else 0
        if L == 1 or N < L * LANE_MIN:
            return self.tile_forward(x, plan, out)
        self._check_in(x, plan.inp.size)
        y = self._out(out, N)
        bounds = [N * i // L for i in range(L + 1)]
        cur = torch.cuda.current_stream(self.device)
        for i, st in enumerate(self._lane_streams, start=1):
            st.wait_stream(cur)  # fork: inputs produced / outputs free on the current stream
            lo, hi = bounds[i], bounds[i + 1]
            with torch.cuda.stream(st):
                self._lanes[i - 1].tile_forward(x[lo:hi], plan, y[lo:hi])
        self.tile_forward(x[:bounds[1]], plan, y[:bounds[1]])
        for st in self._lane_streams:
            cur.wait_stream(st)  # join: later work on the current stream (incl. reuse of x / y) follows
        return y

    __call__ = forward

    def forward_async(self, x: torch.Tensor, out: torch.Tensor, on_lane=None, pre_lane=None) -> torch.Tensor:
        """Throughput form of :meth:`forward` for a loop of forwards on the same buffers.

        Each lane enqueues its slice on its own stream and is NOT joined back: consecutive calls
        pipeline instead of being realigned by a join every call. When every lane is idle (the first
        call, or after any device synchronisation) the lanes fork from the current stream; with
        ``stagger`` set, lane i >= 1 then starts when lane i-1's stage 1 (Conv1 + Pool1) is done, half
        a forward apart (one lane's transforms and pools under the other's GEMMs), else together.

        Contract: ``out`` holds a call's results once :meth:`join` has made the current stream wait
        for the lanes (or after a device synchronisation); ``x`` and ``out`` must not be written by
        other work until then. ``pre_lane(i, lo, hi)`` / ``on_lane(i, lo, hi)``, if given, run with
        lane i's stream current right before / after it enqueues images [lo, hi) (e.g. waiting for a
        collective still reading that output slice / a per-lane collective on it)."""
        L = 1 + len(self._lanes)
        N = self._check_in(x, self.H)
        out = self._out(out, N)
        if L == 1 or N < L * LANE_MIN or not self.is_cuda:
            if pre_lane is not None:
                pre_lane(0, 0, N)
            y = self.forward(x, out)
            if on_lane is not None:
                on_lane(0, 0, N)
            return y
        if self._own_stream is None:
            self._own_stream = torch.cuda.Stream(self.device)
        streams = [self._own_stream, *self._lane_streams]
        engines = [self, *self._lanes]
        plan = full_plan(self.H, self.W, self.b1, self.b2)
        bounds = self.lane_bounds(N)
        fresh = all(st.query() for st in streams)
        cur = torch.cuda.current_stream(self.device)
        ev = None
        for i, (eng, st) in enumerate(zip(engines, streams)):
            lo, hi = bounds[i], bounds[i + 1]
            with torch.cuda.stream(st):
                if fresh:
                    st.wait_stream(cur)  # inputs produced / outputs free on the current stream
                    if ev is not None:
                        st.wait_event(ev)
                if pre_lane is not None:
                    pre_lane(i, lo, hi)
                if fresh and i + 1 < L and self.stagger:
                    eng.stage1(x[lo:hi], plan)  # = tile_forward as stage1 + stage2, with the phase event between
                    ev = torch.cuda.Event()
                    ev.record(st)
                    eng.stage2(hi - lo, plan, out[lo:hi])
                else:
                    eng.tile_forward(x[lo:hi], plan, out[lo:hi])
                if on_lane is not None:
                    on_lane(i, lo, hi)
        return out

    def lane_bounds(self, n: int) -> list[int]:
        """Image boundaries [0, ..., n] of the lanes :meth:`forward_async` runs ``n`` images on."""
        return split_lanes(n, 1 + len(self._lanes) if self.is_cuda else 1)

    def join(self) -> None:
        """Make the current stream wait for every lane of :meth:`forward_async`."""
        if not self.is_cuda:
            return
        cur = torch.cuda.current_stream(self.device)
        for st in ([self._own_stream] if self._own_stream is not None else []) + self._lane_streams:
            cur.wait_stream(st)

    def lane_count(self) -> int:
        return 1 + len(self._lanes)

    def tile_forward(self, x: torch.Tensor, tile: TilePlan, out: torch.Tensor | None = None) -> torch.Tensor:
        """Row tile: ``x`` holds input rows ``tile.inp`` of N images; returns output rows ``tile.out``."""
        N = self._check_in(x, tile.inp.size)
        y = self._out(out, N, tile.out.size)
        if tile.out.size == 0 or N == 0:
            return y
        self._ensure(N)
        if self.is_cuda:
            nat.call("anx_engine_tile_forward", self._engine, x.data_ptr(), N, C.byref(_tile_c(tile)), y.data_ptr(),
                     self._stream())
        else:
            nat.call("anx_cpu_engine_tile_forward", self._engine, x.data_ptr(), N, C.byref(_tile_c(tile)),
                     y.data_ptr())
        return y

    def stage1(self, x: torch.Tensor, tile: TilePlan) -> None:
        """conv1+ReLU+pool1 of input rows ``tile.inp`` into the conv2 input window (rows tile.p1)."""
        N = self._check_in(x, tile.inp.size)
        self._ensure(N)
        if self.is_cuda:
            nat.call("anx_engine_stage1", self._engine, x.data_ptr(), N, C.byref(_tile_c(tile)), self._stream())
        else:
            nat.call("anx_cpu_engine_stage1", self._engine, x.data_ptr(), N, C.byref(_tile_c(tile)))

    def stage2(self, N: int, tile: TilePlan, out: torch.Tensor | None = None) -> torch.Tensor:
        """conv2+ReLU+pool2+LRN of the (halo-completed) window -> output rows ``tile.out``."""
        y = self._out(out, N, tile.out.size)
        if tile.out.size == 0 or N == 0:
            return y
        if self.is_cuda:
            nat.call("anx_engine_stage2", self._engine, N, C.byref(_tile_c(tile)), y.data_ptr(), self._stream())
        else:
            nat.call("anx_cpu_engine_stage2", self._engine, N, C.byref(_tile_c(tile)), y.data_ptr())
        return y

    # ------------------------------------------------------------------ conv2 input window (halo slots)
    def window_rows_shape(self, N: int, rows: int) -> tuple[int, int, int, int]:
        return (N, rows, self.dims.Wp1 + 2 * self.b2.conv.P, self.dims.C1)

    def _window_geom(self, tile: TilePlan, r: int):
        p = C.c_void_p()
        row, img = C.c_size_t(), C.c_size_t()
        fn = "anx_engine_window" if self.is_cuda else "anx_cpu_engine_window"
        nat.call(fn, self._engine, C.byref(_tile_c(tile)), 0, r, C.byref(p), C.byref(row), C.byref(img))
        return p.value, row.value, img.value

    def _copy2d(self, dst, dpitch, src, spitch, width, height):
        if self.is_cuda:
            nat.call("anx_memcpy2d_async", dst, dpitch, src, spitch, width, height, self._stream())
        else:
            nat.call("anx_memcpy2d_host", dst, dpitch, src, spitch, width, height)

    def window_put(self, tile: TilePlan, lo: int, src: torch.Tensor) -> None:
        """Write pool1 rows [lo, lo+src.shape[1]) (full padded rows, [N,rows,Wq,C1]) into the conv2
        input window of ``tile`` — the receive side of a halo exchange."""
        N, rows = src.shape[0], src.shape[1]
        if rows == 0 or N == 0:
            return
        if not (tile.q.lo <= lo and lo + rows <= tile.q.hi):
            raise ValueError("halo rows outside the tile's conv2 window")
        src = src.contiguous()
        base, row_f, img_f = self._window_geom(tile, lo)
        self._copy2d(base, img_f * 4, src.data_ptr(), rows * row_f * 4, rows * row_f * 4, N)

    def window_get(self, tile: TilePlan, lo: int, hi: int, N: int) -> torch.Tensor:
        """Copy pool1 rows [lo, hi) of the window out as [N, hi-lo, Wq, C1] (the send side)."""
        dst = torch.empty(self.window_rows_shape(N, hi - lo), device=self.device)
        if hi <= lo or N == 0:
            return dst
        base, row_f, img_f = self._window_geom(tile, lo)
        self._copy2d(dst.data_ptr(), (hi - lo) * row_f * 4, base, img_f * 4, (hi - lo) * row_f * 4, N)
        return dst
