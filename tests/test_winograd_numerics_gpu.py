"""fp32 Winograd kernels at realistic dynamic range (randn activations, He-init weights), with the
error bounded relative to the sum of absolute products Σ|x·w| of each output — the scale of fp32
accumulation error itself (a direct fp32 conv sits at ~1e-7 of it). The reference-init tests (inputs
U[0,0.1), weights ±0.01) exercise a narrow range only; these pin the transforms' cancellation error.
Also: the exact bench.py step (stream lanes) against the fp64 oracle, images of every lane."""
import math

import pytest
import torch

from anx import _native as nat
from anx.models.alexnet_blocks import AlexNetBlocks
from anx.models.reference import blocks_forward, blocks_forward_all, conv2d_nhwc

pytestmark = pytest.mark.gpu
# Bounds relative to Σ|x·w| per output. F(3x3,5x5) (Conv2) interpolates at 7 points (0, ±1, ±2, ±1/2)
# and F(3x3,3x3) (Conv1 polyphase) at 5, so the transforms cancel more for Conv2. MI355X run: Conv2
# max 1.8-2.6e-6 (mean 8e-8), Conv1 max 1.0-1.3e-6 (mean 4.4e-8). A broken transform or fold is >=1e-3.
# F(4x4,5x5) (8 points, {0, +-1, +-2, +-1/2, inf}) sits ~1.3x above F(3,5) in tools/winograd_numerics.py.
BOUND_CONV2 = 1e-5
BOUND_CONV1 = 4e-6


def _rel_to_terms(y, x, w, b, S, P, groups=1):
    ref = conv2d_nhwc(x.double(), w.double(), b.double(), S, P, groups)
    terms = conv2d_nhwc(x.double().abs(), w.double().abs(), b.double().abs(), S, P, groups)
    rel = (y.double() - ref).abs() / (terms + 1e-30)
    print(f"error / sum|x*w|: max {rel.max().item():.3e} mean {rel.mean().item():.3e}")
    return rel.max().item()


@pytest.mark.parametrize("N,groups,tile", [(12, 1, 3), (12, 2, 3), (9, 1, 3), (128, 1, 3), (140, 2, 3), (12, 1, 4),
                                          (9, 1, 4), (128, 1, 4), (141, 1, 4)])
def test_conv2_winograd_randn_he(cuda, N, groups, tile):
    """Conv2 (31x31 padded window, 96 -> 256, 5x5): randn inputs, He-normal weights; Winograd F(3x3,5x5)
    and F(4x4,5x5) (wino_gemm16.hpp: 16x16x4 MFMAs, 4x4 output tiles with a clipped last row/column)."""
    torch.manual_seed(21 + N)
    C, K = 96, 256
    x = torch.randn(N, 31, 31, C, device=cuda)
    x[:, :2] = 0
    x[:, -2:] = 0
    x[:, :, :2] = 0
    x[:, :, -2:] = 0  # the zero border of the conv2 window
    w = torch.randn(K, C // groups, 5, 5) * math.sqrt(2.0 / (C // groups * 25))
    b = torch.randn(K, device=cuda) * 0.1
    y = torch.full((N, 27, 27, K), float("nan"), device=cuda)
    nat.call("anx_conv2_wino_tile", x.data_ptr(), N, 31, 31, C, w.contiguous().data_ptr(), K, groups, b.data_ptr(),
             y.data_ptr(), 0, nat.stream_ptr(cuda), tile)
    assert torch.isfinite(y).all()
    assert _rel_to_terms(y, x, w.to(cuda), b, 1, 0, groups) < BOUND_CONV2


@pytest.mark.parametrize("N", [5, 70])
def test_conv1_polyphase_winograd_randn_he(cuda, N):
    """Conv1 (227x227x3, 11x11/4, 96 filters) on the polyphase Winograd path: randn inputs."""
    torch.manual_seed(31 + N)
    x = torch.randn(N, 227, 227, 3, device=cuda)
    w = torch.randn(96, 3, 11, 11) * math.sqrt(2.0 / (3 * 121))
    b = torch.randn(96, device=cuda) * 0.1
    y = torch.full((N, 55, 55, 96), float("nan"), device=cuda)
    nat.call("anx_conv1_wino", x.data_ptr(), N, 227, 227, w.contiguous().data_ptr(), 96, 11, b.data_ptr(),
             y.data_ptr(), 0, nat.stream_ptr(cuda))
    assert torch.isfinite(y).all()
    assert _rel_to_terms(y, x, w.to(cuda), b, 4, 0) < BOUND_CONV1


@pytest.mark.parametrize("tile", [3, 4])
def test_full_blocks_randn_he_vs_oracle(cuda, tile):
    """The whole Blocks 1-2 engine (both Winograd convs, pools, LRN) at randn/He scale, Conv2 on either
    Winograd tile (Knobs::conv2_tile)."""
    torch.manual_seed(5)
    w1 = torch.randn(96, 3, 11, 11) * math.sqrt(2.0 / 363)
    w2 = torch.randn(256, 96, 5, 5) * math.sqrt(2.0 / 2400)
    ws = {"w1": w1, "b1": torch.randn(96) * 0.1, "w2": w2, "b2": torch.randn(256) * 0.1}
    m = AlexNetBlocks(ws, device=cuda, max_batch=24, knobs={"conv2_tile": tile})
    assert m.get_knob("conv2_tile") == tile
    x = torch.randn(24, 227, 227, 3)
    y = m(x.to(cuda)).cpu().double()
    ref = blocks_forward(x, m.weights, m.b1, m.b2)
    assert (y - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_bench_step_vs_oracle(cuda):
    """bench.py's default step: 128 images as 2 stream lanes of 64 (one engine per HIP stream),
    checked against the fp64 oracle on images from both lanes including the first and last."""
    B = 128
    m = AlexNetBlocks(init="rand", seed=1234, device=cuda, max_batch=B, lanes=2)
    g = torch.Generator(device=cuda)
    g.manual_seed(1234)
    x = torch.rand((B, 227, 227, 3), device=cuda, generator=g) * 0.1
    y = m(x)
    ref = blocks_forward_all(x, m.weights, m.b1, m.b2, device=cuda)  # all 128 images, fp64
    err = (y.cpu().double() - ref).abs().amax(dim=(1, 2, 3)) / ref.abs().amax(dim=(1, 2, 3))
    assert err.max().item() <= 1e-5, (err.argmax().item(), err.max().item())
    # the second lane's half is bitwise what one engine computes for it alone
    solo = AlexNetBlocks(init="rand", seed=1234, device=cuda, max_batch=B // 2)
    assert torch.equal(solo(x[B // 2:].contiguous()), y[B // 2:])
