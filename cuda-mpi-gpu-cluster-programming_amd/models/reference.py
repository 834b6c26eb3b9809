"""Pure-PyTorch oracle of AlexNet Blocks 1-2 (NHWC in / NHWC out).

Used only to check the native kernels ("numeric unit tests per kernel vs CPU reference
and vs PyTorch-ROCm"). Runs on any device/dtype; tests use float64 on the CPU.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..config import BLOCK1, BLOCK2, BlockSpec


def conv2d_nhwc(x, w, b, S, P, groups=1, relu=False):
    y = F.conv2d(x.permute(0, 3, 1, 2), w, b, stride=S, padding=P, groups=groups)
    if relu:
        y = torch.relu(y)
    return y.permute(0, 2, 3, 1).contiguous()


def maxpool_nhwc(x, Fp, Sp):
    return F.max_pool2d(x.permute(0, 3, 1, 2), Fp, Sp).permute(0, 2, 3, 1).contiguous()


def lrn_nhwc(x, size, alpha, beta, k, mode="div_n"):
    a = alpha if mode == "div_n" else alpha * size  # torch divides alpha by size internally
    return F.local_response_norm(x.permute(0, 3, 1, 2), size, alpha=a, beta=beta, k=k).permute(0, 2, 3, 1).contiguous()


def blocks_forward(x, weights, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2, dtype=torch.float64):
    """x: [N,H,W,3] -> [N,Hp2,Wp2,K2]. ``weights``: {w1,b1,w2,b2} KCFF tensors."""
    dev = x.device
    cast = lambda t: t.to(device=dev, dtype=dtype)  # noqa: E731
    h = cast(x)
    h = conv2d_nhwc(h, cast(weights["w1"]), cast(weights["b1"]), b1.conv.S, b1.conv.P, b1.conv.groups, relu=True)
    h = maxpool_nhwc(h, b1.pool.F, b1.pool.S)
    if b1.has_lrn:
        h = lrn_nhwc(h, b1.lrn.N, b1.lrn.alpha, b1.lrn.beta, b1.lrn.k, b1.lrn.mode)
    h = conv2d_nhwc(h, cast(weights["w2"]), cast(weights["b2"]), b2.conv.S, b2.conv.P, b2.conv.groups, relu=True)
    h = maxpool_nhwc(h, b2.pool.F, b2.pool.S)
    if b2.has_lrn:
        h = lrn_nhwc(h, b2.lrn.N, b2.lrn.alpha, b2.lrn.beta, b2.lrn.k, b2.lrn.mode)
    return h


def blocks_forward_all(x, weights, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2, device=None, chunk: int = 64):
    """The fp64 oracle of EVERY image of a batch, ``chunk`` images at a time on ``device`` (the GPU in
    the GPU tests: fp64 convolutions run there as im2col + DGEMM in seconds where the CPU takes
    minutes), returned on the CPU. The tests check whole batches with it, not samples."""
    dev = torch.device(device) if device is not None else x.device
    outs = [blocks_forward(x[i:i + chunk].to(dev), weights, b1, b2).cpu() for i in range(0, x.shape[0], chunk)]
    return torch.cat(outs)
