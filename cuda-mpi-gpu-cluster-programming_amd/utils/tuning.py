"""Kernel selection knobs of the native engines (anx/knobs.hpp), per engine.

Every :class:`~anx.models.alexnet_blocks.AlexNetBlocks` / :class:`~anx.models.alexnet_full.AlexNetFull`
owns its knobs (``knobs={...}`` at construction, ``set_knob`` later); nothing here is process-wide.
Names and values:

* ``conv2_algo``: Conv2 (5x5, stride 1) on the MFMA path — ``auto`` (Winograd F(3x3,5x5) when
  eligible and the launch exceeds 8 images), ``direct`` (implicit GEMM; bit-identical across any row
  decomposition), ``winograd``.
* ``conv1_algo``: Conv1 (11x11, stride 4) — ``auto``/``winograd`` (polyphase Winograd F(3x3,3x3)) or
  ``direct``.
* integer knobs: ``chunk1``, ``chunk2`` (images per launch), ``conv1_occ``, ``conv2_occ`` (Winograd
  GEMM workgroups-per-CU caps), ``force_vec4``, ``force_scalar`` (direct GEMM tiles), and the bf16
  full model's ``bf16_glds``, ``bf16_big``, ``bf16_lrn_tile``, ``bf16_fc_cfg``,
  ``bf16_fc_minkt``, ``bf16_conv1`` (2, the default: Conv1 as the persistent row-band kernel reading
  the fp32 image; 1: the same kernel on the s2d4 polyphase copy; 0: s2d4 + the implicit-GEMM tiles),
  ``bf16_pool1`` (1, the default: pool1 in the row-band kernel's epilogue when each image has its own
  workgroup; 0: Conv1 writes its map and maxpool_bf16 follows); ``conv1_band`` (2, the default: the
  Conv1 input transform stages a tile row's image rows in LDS, all 4 phase rows x half the tile
  columns per workgroup; 1: 2 phase rows x all columns; 0: per-tile global gathers);
  ``fuse_pool1`` (1, the
  default: a tile that computes all the pool1 rows its conv2 window needs runs pool1 inside the
  Winograd input transform; 0: the pool1 kernel and the window buffer); ``conv1_sub`` / ``conv2_sub``
  (images per Conv1 / Conv2 transform + GEMM launch pair inside a fused forward; 0 = whole launch: a
  small sub-chunk rewrites the V workspace in place, inside the Infinity Cache); ``conv1_fused`` (1, the
  default: Conv1 as one kernel, the polyphase input transform built in LDS inside the Winograd GEMM;
  0: the band transform kernel + GEMM); ``conv1_pool`` (1, the default: pool1 in that kernel's epilogue for
  whole images, the conv1 map never reaches HBM; 0: Conv1 writes its map and the input transform pools it);
  ``conv2_pool`` (1, the default since round 6: pool2 in the F(4x4,5x5) GEMM's epilogue for whole images, the
  27x27 map never reaches HBM, +3 % on the bench step with the hand-scheduled GEMM; 0: the GEMM writes its map
  and the pool2 + LRN kernel pools it);
  ``conv2_tile`` (Conv2's Winograd output tile: 3 = F(3x3,5x5), 4 = F(4x4,5x5), 21 % fewer multiplies);
  ``conv2_sched`` (1, the default: the F(4x4,5x5) GEMM's hand-scheduled K slice, bitwise equal to 0, the
  compiler's schedule); ``lrn_wgs`` (256, the default: grid cap of the pool2-merge + LRN kernel, its waves
  walking the remaining pixels; 0 = one wave per pixel pair; same bits).
"""
from __future__ import annotations

import ctypes as C

from .. import _native as nat

ALGOS = {"auto": 0, "direct": 1, "winograd": 2}
KNOBS = ("conv1_algo", "conv2_algo", "chunk1", "chunk2", "force_vec4", "force_scalar", "bf16_glds", "bf16_big",
         "bf16_lrn_tile", "bf16_conv1", "bf16_pool1", "bf16_fc_cfg", "bf16_fc_minkt", "conv1_occ", "conv2_occ", "conv1_band", "fuse_pool1", "conv1_sub", "conv2_sub",
         "conv1_fused", "conv1_pool", "conv2_pool", "conv2_tile", "conv2_sched", "conv2_in_pg", "lrn_wgs")


def knob_value(name: str, value) -> int:
    """Normalise a knob value: algorithm names for ``conv*_algo``, ints (or bools) otherwise."""
    if name not in KNOBS:
        raise ValueError(f"unknown knob {name!r}; known: {', '.join(KNOBS)}")
    if name.endswith("_algo") and isinstance(value, str):
        if value not in ALGOS:
            raise ValueError(f"{name} must be one of {sorted(ALGOS)}")
        return ALGOS[value]
    return int(value)


def default_knob(name: str) -> int:
    """The value a new engine starts from (built-in default or its ANX_* environment override)."""
    knob_value(name, 0)
    v = C.c_int()
    nat.call("anx_default_knob", name.encode(), C.byref(v))
    return v.value


def apply_knobs(handle, knobs: dict | None, full: bool = False) -> None:
    """Set ``knobs`` on one native engine handle (BlocksEngine, or FullEngine with ``full``)."""
    fn = "anx_full_set_knob" if full else "anx_engine_set_knob"
    for k, v in (knobs or {}).items():
        nat.call(fn, handle, k.encode(), knob_value(k, v))


def read_knob(handle, name: str, full: bool = False) -> int:
    v = C.c_int()
    knob_value(name, 0)
    nat.call("anx_full_get_knob" if full else "anx_engine_get_knob", handle, name.encode(), C.byref(v))
    return v.value
