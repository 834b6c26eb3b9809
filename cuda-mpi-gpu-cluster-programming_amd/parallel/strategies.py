"""Distributed forward strategies for AlexNet Blocks 1-2.

  * :func:`replicate_forward`  — P1 "broadcast-all" (V2.1, v2_mpi_only/2.1_broadcast_all/src/main.cpp:49-85):
    every rank computes the whole batch; rank 0's result is the answer (no gather, as the reference).

The row decomposition (P2: V2.2, V4, V5) and the image split (P6) run on the native runtimes
(``anx/v4.hpp``, ``anx/v5.hpp`` through :mod:`anx.parallel.workloads`; CPU ranks: the V5 runtime in
host mode), the pipelined data-parallel form on :class:`anx.parallel.pipeline.ScatterComputeGather`,
and the filter split (P7) on :func:`anx.parallel.tensor.filter_parallel_forward`.
"""
from __future__ import annotations

import torch

from ..utils.timer import PhaseTimer


def replicate_forward(model, x: torch.Tensor, timer: PhaseTimer | None = None):
    timer = timer or PhaseTimer(model.device, sync=False)
    with timer.phase("compute"):
        y = model(x)
    return y


__all__ = ["replicate_forward"]
