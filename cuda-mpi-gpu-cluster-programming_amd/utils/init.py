"""Deterministic parameter/input initialisation (bit-identical to csrc/include/anx/rng.hpp).

Two modes, as in the reference:
  * ``const`` — input 1.0, all weights 0.01, biases 0 (v2..v4 mains, e.g.
    final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:28-34): reproduces the golden outputs
    44.4147 / 29.2931 ....
  * ``rand`` — input U[0,1)*0.1, weights (U-0.5)*0.02, biases 0.1
    (v1_serial/src/alexnet_serial.cpp:39-57) from a counter-based splitmix64 stream, so the
    same (seed, stream, index) gives the same value in C++, numpy or on any rank.
"""
from __future__ import annotations

import numpy as np
import torch

from ..config import BLOCK1, BLOCK2, BlockSpec, IN_C, IN_H, IN_W

STREAM_INPUT, STREAM_W1, STREAM_B1, STREAM_W2, STREAM_B2, STREAM_EXTRA = 0, 1, 2, 3, 4, 8

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, stream: int, n: int, offset: int = 0) -> np.ndarray:
    """float32 U[0,1) values for indices offset..offset+n-1 of (seed, stream)."""
    key = ((np.uint64(seed) << np.uint64(32)) & _M) ^ ((np.uint64(stream) << np.uint64(56)) & _M)
    i = np.arange(offset, offset + n, dtype=np.uint64)
    bits = _splitmix64(i ^ key) >> np.uint64(40)
    return (bits.astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def conv_weight_shape(spec: BlockSpec) -> tuple[int, int, int, int]:
    c = spec.conv
    return (c.K, c.C // c.groups, c.F, c.F)


def init_weights(mode: str = "const", seed: int = 0, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2,
                 wv: float = 0.01, bv: float = 0.0) -> dict[str, torch.Tensor]:
    """KCFF weights + biases for Blocks 1-2 as CPU float32 tensors {w1,b1,w2,b2}."""
    s1, s2 = conv_weight_shape(b1), conv_weight_shape(b2)
    n1, n2 = int(np.prod(s1)), int(np.prod(s2))
    if mode == "const":
        w1 = np.full(n1, wv, np.float32)
        w2 = np.full(n2, wv, np.float32)
        bb1 = np.full(b1.conv.K, bv, np.float32)
        bb2 = np.full(b2.conv.K, bv, np.float32)
    elif mode == "rand":
        w1 = (uniform(seed, STREAM_W1, n1) - np.float32(0.5)) * np.float32(0.02)
        w2 = (uniform(seed, STREAM_W2, n2) - np.float32(0.5)) * np.float32(0.02)
        bb1 = np.full(b1.conv.K, 0.1, np.float32)
        bb2 = np.full(b2.conv.K, 0.1, np.float32)
    else:
        raise ValueError(f"unknown init mode {mode!r}")
    return {
        "w1": torch.from_numpy(w1.reshape(s1)),
        "b1": torch.from_numpy(bb1),
        "w2": torch.from_numpy(w2.reshape(s2)),
        "b2": torch.from_numpy(bb2),
    }


def init_input(N: int = 1, mode: str = "const", seed: int = 0, H: int = IN_H, W: int = IN_W, C: int = IN_C,
               first_image: int = 0) -> torch.Tensor:
    """NHWC float32 CPU input. In ``rand`` mode image j of the global batch is identical on every
    rank (indices are global), so a rank can synthesise just its shard (``first_image``)."""
    per = H * W * C
    if mode == "const":
        x = np.ones(N * per, np.float32)
    elif mode == "rand":
        x = uniform(seed, STREAM_INPUT, N * per, offset=first_image * per) * np.float32(0.1)
    else:
        raise ValueError(f"unknown init mode {mode!r}")
    return torch.from_numpy(x.reshape(N, H, W, C))


def init_input_device(N: int, seed: int, device, H: int = IN_H, W: int = IN_W, C: int = IN_C,
                      first_image: int = 0) -> torch.Tensor:
    """Same values as ``init_input(mode='rand')`` generated directly on the device (large batches)."""
    per = H * W * C
    out = torch.empty(N * per, dtype=torch.float32, device=device)
    chunk = 1 << 24
    for s in range(0, N * per, chunk):
        e = min(N * per, s + chunk)
        host = uniform(seed, STREAM_INPUT, e - s, offset=first_image * per + s) * np.float32(0.1)
        out[s:e].copy_(torch.from_numpy(host), non_blocking=False)
    return out.view(N, H, W, C)
