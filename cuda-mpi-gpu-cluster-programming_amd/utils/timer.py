"""Phase timers and roctx ranges.

The reference times whole runs with ``std::chrono`` around context creation, mallocs and copies
(v3_cuda_only/src/main_cuda.cpp:30-35, v4_mpi_cuda/src/main_mpi_cuda.cpp:151-160).
Here every phase (bcast, scatter, halo, h2d, compute, d2h, gather) is timed on a monotonic clock,
optionally fenced by a device synchronize so the split is exact, and wrapped in a roctx range so
rocprofv3 ``--marker-trace`` shows the same phases on the timeline.
"""
from __future__ import annotations

import ctypes
import time
from collections import OrderedDict
from contextlib import contextmanager

import torch

_roctx = None


def _rx():
    global _roctx
    if _roctx is None:
        _roctx = False
        for name in ("libroctx64.so.4", "libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx or None


@contextmanager
def roctx_range(name: str):
    lib = _rx()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class PhaseTimer:
    """Accumulates wall time per named phase. ``sync=True`` fences each phase with a device
    synchronize (exact split; use for breakdowns, not for headline throughput)."""

    def __init__(self, device=None, sync: bool = True):
        self.device = torch.device(device) if device is not None else None
        self.sync = sync and self.device is not None and self.device.type == "cuda"
        self.ms: "OrderedDict[str, float]" = OrderedDict()

    def _fence(self):
        if self.sync:
            torch.cuda.synchronize(self.device)

    @contextmanager
    def phase(self, name: str):
        self._fence()
        t0 = time.perf_counter()
        with roctx_range(name):
            yield
        self._fence()
        self.ms[name] = self.ms.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def total(self) -> float:
        return sum(self.ms.values())

    def scaled(self, k: float) -> dict:
        return {n: v * k for n, v in self.ms.items()}
