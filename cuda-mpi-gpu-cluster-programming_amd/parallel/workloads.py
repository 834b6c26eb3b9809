"""The reference's multi-GPU programs as steady-state, strong-scaling benchmark steps
(``bench.py --workload v4|v5``).

The reference's V4 (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:52-130) keeps the batch on rank
0's host, scatters input rows, runs the tile forward and gathers output rows back to the host; its
planned V5 (README.md:157-166) keeps every byte on the device and exchanges per-layer halos between
GPUs.

* :class:`NativeV5` / :class:`NativeV4` — the GPU programs: thin clients of the native runtimes
  (``anx/v5.hpp`` / ``anx/v4.hpp`` through ``libanx_dist``'s C ABI). The runtimes own the plan, the
  buffers, the streams and the transport (RCCL over xGMI; the RCCL transport over the loopback device
  comm, or the peer IPC transport with device-side flags, when ranks share a GPU); Python only passes
  the job shape and the root's weights / batch and reads back the output, the phase times and the
  layout. The V5 transfer list is :func:`anx.parallel.plan.step_schedule` exactly
  (tests/test_v5_runtime.py). Default row split: the native cost model's pick (anx/cost.hpp).
* CPU ranks (``bench.py --device cpu``, tests/test_dist_cpu.py) run the SAME native V5 runtime in
  host mode (``impl="host"``): the host engine and the host transport over the runtime's own TCP
  channel, with the layout, schedule and halo chunks the GPU ranks use. V4 on CPU is the overlap-tile
  layer with the batch scattered from the root every step. There is no second, Python-level
  implementation of the scatter / halo / gather::

    v4  root host --H2D--> root device --scatter (images x input rows incl. halo)--> ranks
        --tile_forward (overlap tiles: no mid-network exchange)--> gather --D2H--> root host
    v5  root --scatter--> ranks --stage1 (conv1+pool1)--> pool1-halo exchange inside each row group
        (per_layer tiles) --stage2 (conv2+pool2+LRN)--> gather --> root
"""
from __future__ import annotations

import torch

import ctypes as C
import json
import os
import socket

from .. import _native as nat
from ..config import BLOCK1, BLOCK2, blocks_dims
from .comm import world
from .plan import OVERLAP, PER_LAYER

# -1: the cost model's pick (anx/cost.hpp); None: rows over every rank; rows2: 2-way row groups (the
# halo exchange on at any even rank count: bench.py's v5 sub-records)
V5_DECOMPS = {"auto": -1, "rows": None, "hybrid": 0, "batch": 1, "rows2": 2}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(port):
    """rank, world, local rank / world, nodes and the runtime's rendezvous port (chosen by rank 0 and
    shared over torch.distributed when it is initialised, else `port` / ANX_V5_PORT)."""
    import torch.distributed as tdist
    up = tdist.is_available() and tdist.is_initialized()
    if up:
        rank, size = world()
    else:  # a launcher's environment (torchrun / anxrun) without a torch process group
        rank, size = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", size))
    nnodes = max(1, size // max(1, local_world))
    if port is None:
        port = int(os.environ.get("ANX_V5_PORT", "0")) or (_free_port() if rank == 0 else 0)
        if size > 1 and up:
            box = [port]
            tdist.broadcast_object_list(box, src=0)
            port = box[0]
        elif size > 1 and not os.environ.get("ANX_V5_PORT"):
            raise ValueError("a native runtime at world > 1 needs torch.distributed, `port` or ANX_V5_PORT")
    return rank, size, local_rank, local_world, nnodes, port


def _root_weights(rank, weights):
    if rank != 0:
        return [None] * 4, None
    if weights is None:
        raise ValueError("rank 0 needs the weights")
    w = {k: weights[k].detach().to("cpu", torch.float32).contiguous() for k in ("w1", "b1", "w2", "b2")}
    return [w[k].data_ptr() for k in ("w1", "b1", "w2", "b2")], w


class NativeV5:
    """V5 on GPUs through the native runtime (one instance per rank; construction is collective).

    ``weights``: rank 0's dict w1/b1/w2/b2 (fp32 KCFF, any device; other ranks may pass None: the
    runtime broadcasts rank 0's device copy over the transport). The rendezvous port of the runtime's
    own bootstrap channel is chosen by rank 0 and shared over torch.distributed when it is
    initialised (else ``port`` / ANX_V5_PORT).
    """

    def __init__(self, batch: int, weights: dict | None, *, specs=(BLOCK1, BLOCK2), H: int = 227, W: int = 227,
                 decomp: str = "auto", layer: str = PER_LAYER, transport: str = "auto", chunks: int = 0,
                 pipeline: int = -1, poison: bool = False, impl: str = "mfma", peer_sync: str = "",
                 port: int | None = None, timeout_s: float = 300.0, input_source: str = "local", lanes: int = 0,
                 keep_log: bool = False, root_images: int = -1):
        if decomp not in V5_DECOMPS:
            raise ValueError(f"decomp must be one of {sorted(V5_DECOMPS)}")
        if layer not in (OVERLAP, PER_LAYER):
            raise ValueError("layer must be overlap or per_layer")
        if input_source not in ("local", "root"):
            raise ValueError("input_source must be local or root")
        if impl not in ("mfma", "direct", "host"):
            raise ValueError("impl must be mfma, direct or host (CPU ranks: host engine + host transport)")
        self.rank, self.world, local_rank, local_world, nnodes, port = _launch(port)
        self.batch, self.b1, self.b2, self.H, self.W = batch, specs[0], specs[1], H, W
        self.dims = blocks_dims(H, W, *specs)
        rw = V5_DECOMPS[decomp]
        rw = self.world if rw is None else rw
        ptrs, self._w = _root_weights(self.rank, weights)
        h = C.c_void_p()
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1").encode()
        nat.dist_call("anx_v5_create", C.byref(h), self.rank, self.world, local_rank, local_world, nnodes, addr, port,
                      timeout_s, C.byref(nat.block_c(self.b1)), C.byref(nat.block_c(self.b2)), H, W, *ptrs, batch, rw,
                      1 if layer == PER_LAYER else 0, transport.encode(), chunks, pipeline, int(poison),
                      {"mfma": 0, "direct": 1, "host": 2}[impl], peer_sync.encode(), 1 if input_source == "root" else 0, lanes,
                      int(keep_log), root_images)
        self._h = h
        self.version, self.layer, self.input_source = "v5", layer, input_source

    # ------------------------------------------------------------------ data
    def fill(self, x: torch.Tensor | None) -> None:
        """Collective: rank 0's global batch [B,H,W,C0] (any device) becomes the input of the following
        steps; other ranks pass None (or anything: ignored)."""
        if self.rank == 0:
            xs = x.detach().to("cpu", torch.float32).contiguous()
            if tuple(xs.shape) != (self.batch, self.H, self.W, self.dims.C0):
                raise ValueError(f"expected [{self.batch},{self.H},{self.W},{self.dims.C0}], got {tuple(xs.shape)}")
            nat.dist_call("anx_v5_set_input", self._h, xs.data_ptr())
        else:
            nat.dist_call("anx_v5_set_input", self._h, None)

    def output(self) -> torch.Tensor | None:
        """Rank 0: the gathered output of the last step (host fp32 [B, Hp2, Wp2, C2])."""
        if self.rank != 0:
            return None
        d = self.dims
        y = torch.empty((self.batch, d.Hp2, d.Wp2, d.C2), dtype=torch.float32)
        nat.dist_call("anx_v5_output", self._h, y.data_ptr())
        return y

    # ------------------------------------------------------------------ steps
    def step(self, record: bool = False, steps: int = 1) -> None:
        nat.dist_call("anx_v5_step", self._h, steps)

    def sync(self) -> None:
        nat.dist_call("anx_v5_sync", self._h)

    def _json(self, name, *extra) -> dict:
        buf = C.create_string_buffer(1 << 16)
        nat.dist_call(name, self._h, buf, len(buf), *extra)
        return json.loads(buf.value.decode())

    def transfer_log(self) -> list[str]:
        """Every transfer this rank's transport issued since construction (``keep_log=True``)."""
        buf = C.create_string_buffer(1 << 22)
        nat.dist_call("anx_v5_log", self._h, buf, len(buf))
        return [l for l in buf.value.decode().splitlines() if l]

    def phase_ms(self, reset: bool = False) -> dict:
        """Mean ms per step since the last reset on the compute stream's critical path (syncs)."""
        return {k: round(v, 4) for k, v in self._json("anx_v5_phases", int(reset)).items()}

    def reset_phases(self) -> None:
        self.phase_ms(reset=True)

    def describe(self) -> dict:
        return {"workload": "v5", "runtime": "native (anx/v5.hpp via libanx_dist)", **self._json("anx_v5_describe")}

    def close(self) -> None:
        if getattr(self, "_h", None):
            nat.dist_call("anx_v5_destroy", self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass


def native_schedule(np_: int, batch: int, row_ways: int = -1, layer: str = PER_LAYER, chunks: int = 0,
                    rank: int = -1, transport: str = "rccl", specs=(BLOCK1, BLOCK2), H: int = 227,
                    W: int = 227, input_source: str = "root") -> list[str]:
    """The native runtime's record-only schedule (no GPU): rank < 0 -> every transfer of one step in
    issue order; else what rank `rank`'s transport issues."""
    buf = C.create_string_buffer(1 << 22)
    nat.check(nat.dist().anx_v5_schedule(np_, C.byref(nat.block_c(specs[0])), C.byref(nat.block_c(specs[1])), H, W,
                                         batch, row_ways, 1 if layer == PER_LAYER else 0, chunks, rank,
                                         transport.encode(), 1 if input_source == "root" else 0, buf, len(buf)),
              "anx_v5_schedule")
    return [l for l in buf.value.decode().splitlines() if l]


class NativeV4:
    """V4 on GPUs through the native host-staged runtime (anx/v4.hpp; construction is collective):
    the batch and the output live in one shared pinned host segment, every rank DMAs its own images x
    input rows (halo included) from it and its output rows back, chunked so H2D / compute / D2H
    overlap.

    ``x_host`` / ``y_host`` are zero-copy views of the segment, valid until :meth:`close`: ``close``
    unmaps it, after which the properties raise and any view or slice kept from them points at
    unmapped memory (take ``.clone()`` of what must outlive the runtime; :meth:`output` does)."""

    def __init__(self, batch: int, weights: dict | None, *, specs=(BLOCK1, BLOCK2), H: int = 227, W: int = 227,
                 decomp: str = "auto", chunks: int = 0, impl: str = "mfma", port: int | None = None,
                 timeout_s: float = 300.0):
        import numpy as np
        if decomp not in V5_DECOMPS:
            raise ValueError(f"decomp must be one of {sorted(V5_DECOMPS)}")
        self.rank, self.world, local_rank, local_world, nnodes, port = _launch(port)
        self.batch, self.b1, self.b2, self.H, self.W = batch, specs[0], specs[1], H, W
        d = self.dims = blocks_dims(H, W, *specs)
        rw = V5_DECOMPS[decomp]
        rw = self.world if rw is None else rw
        ptrs, self._w = _root_weights(self.rank, weights)
        h = C.c_void_p()
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1").encode()
        nat.dist_call("anx_v4_create", C.byref(h), self.rank, self.world, local_rank, local_world, nnodes, addr, port,
                      timeout_s, C.byref(nat.block_c(self.b1)), C.byref(nat.block_c(self.b2)), H, W, *ptrs, batch, rw,
                      chunks, 0 if impl == "mfma" else 1)
        self._h = h
        pin, pout = C.POINTER(C.c_float)(), C.POINTER(C.c_float)()
        nat.dist_call("anx_v4_segment", h, C.byref(pin), C.byref(pout))
        self._x_host = torch.from_numpy(np.ctypeslib.as_array(pin, shape=(batch, H, W, d.C0)))
        self._y_host = torch.from_numpy(np.ctypeslib.as_array(pout, shape=(batch, d.Hp2, d.Wp2, d.C2)))
        self.version, self.layer = "v4", OVERLAP

    @property
    def x_host(self) -> torch.Tensor:
        if self._x_host is None:
            raise RuntimeError("NativeV4 is closed: its shared segment is unmapped")
        return self._x_host

    @property
    def y_host(self) -> torch.Tensor:
        if self._y_host is None:
            raise RuntimeError("NativeV4 is closed: its shared segment is unmapped")
        return self._y_host

    def fill(self, x: torch.Tensor | None) -> None:
        """Collective: rank 0 writes the global batch into the shared segment."""
        if self.rank == 0:
            if tuple(x.shape) != tuple(self.x_host.shape):
                raise ValueError(f"expected {tuple(self.x_host.shape)}, got {tuple(x.shape)}")
            self.x_host.copy_(x.detach().to("cpu", torch.float32))
        nat.dist_call("anx_v4_input_ready", self._h)

    def step(self, record: bool = False, steps: int = 1) -> None:
        nat.dist_call("anx_v4_step", self._h, steps)

    def sync(self) -> None:
        """Collective: every rank's copies are done (the output segment is complete)."""
        nat.dist_call("anx_v4_sync_all", self._h)

    def output(self) -> torch.Tensor | None:
        return self.y_host.clone() if self.rank == 0 else None

    def _json(self, name, *extra) -> dict:
        buf = C.create_string_buffer(4096)
        nat.dist_call(name, self._h, buf, len(buf), *extra)
        return json.loads(buf.value.decode())

    def phase_ms(self, reset: bool = False) -> dict:
        return {k: round(v, 4) for k, v in self._json("anx_v4_phases", int(reset)).items()}

    def reset_phases(self) -> None:
        self.phase_ms(reset=True)

    def describe(self) -> dict:
        return {"workload": "v4", "runtime": "native (anx/v4.hpp via libanx_dist)", **self._json("anx_v4_describe")}

    def probe_h2d_gbps(self, reps: int = 5) -> float:
        """This rank's host link alone: GB/s of one H2D of its whole share (syncs its streams)."""
        v = C.c_double()
        nat.dist_call("anx_v4_probe_h2d", self._h, reps, C.byref(v))
        return v.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._x_host = self._y_host = None
            nat.dist_call("anx_v4_destroy", self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass
