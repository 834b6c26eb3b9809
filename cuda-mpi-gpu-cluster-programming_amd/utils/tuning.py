"""Process-wide kernel selection knobs of the native engine (read at launch time).

* ``set_conv2_algo``: Conv2 (5x5, stride 1) on the MFMA path — ``auto`` (Winograd F(3x3,5x5) when
  eligible), ``direct`` (implicit-GEMM; bit-identical across any row decomposition), ``winograd``,
  ``winograd_unfused`` (separate batched GEMM + output transform; A/B only).
* ``set_conv1_algo``: Conv1 (11x11, stride 4) on the MFMA path — ``auto``/``winograd`` (polyphase
  Winograd F(3x3,3x3)) or ``direct`` (implicit GEMM; bit-identical across any row decomposition).
* ``force_conv_variant``: pin an implicit-GEMM tile variant (A/B tuning; ``None`` = heuristic).
"""
from __future__ import annotations

from contextlib import contextmanager

from .. import _native as nat

_ALGOS = {"auto": 0, "direct": 1, "winograd": 2, "winograd_unfused": 3}


def set_conv2_algo(name: str) -> None:
    if name not in _ALGOS:
        raise ValueError(f"conv2 algo must be one of {sorted(_ALGOS)}")
    nat.call("anx_set_conv2_algo", _ALGOS[name])


def get_conv2_algo() -> str:
    v = nat.lib().anx_get_conv2_algo()
    return {i: k for k, i in _ALGOS.items()}[v]


@contextmanager
def conv2_algo(name: str):
    old = get_conv2_algo()
    set_conv2_algo(name)
    try:
        yield
    finally:
        set_conv2_algo(old)


_ALGOS1 = {"auto": 0, "direct": 1, "winograd": 2}


def set_conv1_algo(name: str) -> None:
    if name not in _ALGOS1:
        raise ValueError(f"conv1 algo must be one of {sorted(_ALGOS1)}")
    nat.call("anx_set_conv1_algo", _ALGOS1[name])


def get_conv1_algo() -> str:
    v = nat.lib().anx_get_conv1_algo()
    return {i: k for k, i in _ALGOS1.items()}[v]


@contextmanager
def conv1_algo(name: str):
    old = get_conv1_algo()
    set_conv1_algo(name)
    try:
        yield
    finally:
        set_conv1_algo(old)


def force_conv_variant(vec4: int | None = None, scalar: int | None = None) -> None:
    nat.call("anx_conv_force_variant", 0, -1 if vec4 is None else vec4)
    nat.call("anx_conv_force_variant", 1, -1 if scalar is None else scalar)
