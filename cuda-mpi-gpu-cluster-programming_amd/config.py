"""Layer specifications and shape algebra (Python mirror of csrc/include/anx/shapes.hpp).

Parity: the reference's ``LayerParams`` bag and dim helpers
(final_project/v1_serial/include/alexnet.hpp:9-24, v4_mpi_cuda/include/alexnet.hpp:28-33) and
the hard-coded hyper-parameters of every version (v1_serial/src/main.cpp:18-43,
v4_mpi_cuda/src/main_mpi_cuda.cpp:146-150).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

IN_H, IN_W, IN_C = 227, 227, 3


def conv_out_dim(d: int, f: int, s: int, p: int) -> int:
    return 0 if (s <= 0 or d + 2 * p < f) else (d + 2 * p - f) // s + 1


def pool_out_dim(d: int, f: int, s: int) -> int:
    return 0 if (s <= 0 or d < f) else (d - f) // s + 1


@dataclass(frozen=True)
class ConvSpec:
    C: int
    K: int
    F: int
    S: int
    P: int
    groups: int = 1


@dataclass(frozen=True)
class PoolSpec:
    F: int = 3
    S: int = 2


@dataclass(frozen=True)
class LrnSpec:
    N: int = 5
    alpha: float = 1e-4
    beta: float = 0.75
    k: float = 2.0
    # "div_n": x / (k + alpha/N * sum)^beta   (V1/V2: v1_serial/src/layers_serial.cpp:152,167)
    # "raw"  : x / (k + alpha * sum)^beta     (V3/V4: v3_cuda_only/src/layers_cuda.cu:138)
    mode: str = "div_n"


@dataclass(frozen=True)
class BlockSpec:
    conv: ConvSpec
    pool: PoolSpec = field(default_factory=PoolSpec)
    has_lrn: bool = False
    lrn: LrnSpec = field(default_factory=LrnSpec)


BLOCK1 = BlockSpec(ConvSpec(3, 96, 11, 4, 0, 1))
BLOCK2 = BlockSpec(ConvSpec(96, 256, 5, 1, 2, 1), has_lrn=True)


def blocks(lrn_mode: str = "div_n", groups2: int = 1) -> tuple[BlockSpec, BlockSpec]:
    """The reference's Blocks 1-2 (groups2=2 gives the AlexNet paper's grouped Conv2)."""
    if lrn_mode not in ("div_n", "raw"):
        raise ValueError("lrn_mode must be 'div_n' or 'raw'")
    b2 = replace(BLOCK2, conv=replace(BLOCK2.conv, groups=groups2), lrn=replace(BLOCK2.lrn, mode=lrn_mode))
    return BLOCK1, b2


@dataclass(frozen=True)
class BlocksDims:
    H: int
    W: int
    C0: int
    H1: int
    W1: int
    C1: int
    Hp1: int
    Wp1: int
    H2: int
    W2: int
    C2: int
    Hp2: int
    Wp2: int


def blocks_dims(H: int = IN_H, W: int = IN_W, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> BlocksDims:
    H1 = conv_out_dim(H, b1.conv.F, b1.conv.S, b1.conv.P)
    W1 = conv_out_dim(W, b1.conv.F, b1.conv.S, b1.conv.P)
    Hp1, Wp1 = pool_out_dim(H1, b1.pool.F, b1.pool.S), pool_out_dim(W1, b1.pool.F, b1.pool.S)
    H2 = conv_out_dim(Hp1, b2.conv.F, b2.conv.S, b2.conv.P)
    W2 = conv_out_dim(Wp1, b2.conv.F, b2.conv.S, b2.conv.P)
    Hp2, Wp2 = pool_out_dim(H2, b2.pool.F, b2.pool.S), pool_out_dim(W2, b2.pool.F, b2.pool.S)
    return BlocksDims(H, W, b1.conv.C, H1, W1, b1.conv.K, Hp1, Wp1, H2, W2, b2.conv.K, Hp2, Wp2)


def flops_per_image(H: int = IN_H, W: int = IN_W, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> float:
    """Multiply-add FLOPs (2 per MAC) of the two convolutions — 1.107 GFLOP for the default."""
    d = blocks_dims(H, W, b1, b2)
    c1 = d.H1 * d.W1 * d.C1 * (b1.conv.C // b1.conv.groups) * b1.conv.F ** 2
    c2 = d.H2 * d.W2 * d.C2 * (b2.conv.C // b2.conv.groups) * b2.conv.F ** 2
    return 2.0 * (c1 + c2)


def mfma_flops_per_image(H: int = IN_H, W: int = IN_W, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2,
                         conv2_tile: int = 4) -> float:
    """FLOPs the matrix cores actually execute per image on the default fp32 path (2 per MAC):
    Conv1 as polyphase Winograd F(3x3,3x3) = ceil(H1/3) x ceil(W1/3) tiles x 25 points x 48
    channels x C1 filters, Conv2 as Winograd F(m x m,5x5) = ceil(H2/m) x ceil(W2/m) tiles x (m+4)^2
    points x C1 x C2 / groups, m = the engine's ``conv2_tile`` (4, the default, for one group of 96
    channels; 3 otherwise). 0.237 GFLOP for the default (0.278 with 3x3 tiles), against 1.107 of direct
    convolution (flops_per_image): the ratio is what the fast algorithms save, and this count (not the
    direct one) is what a matrix-core roofline compares against (157 TF/s fp32 peak)."""
    d = blocks_dims(H, W, b1, b2)
    m = 4 if conv2_tile == 4 and b2.conv.groups == 1 and b2.conv.C == 96 else 3
    c1 = -(-d.H1 // 3) * -(-d.W1 // 3) * 25 * 48 * d.C1
    c2 = -(-d.H2 // m) * -(-d.W2 // m) * (m + 4) ** 2 * (b2.conv.C // b2.conv.groups) * d.C2
    return 2.0 * (c1 + c2)
