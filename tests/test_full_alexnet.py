"""Full-AlexNet bf16 extension: shapes/init on the CPU, logits vs the PyTorch fp32 oracle on the GPU
(bf16 storage of weights and activations: ~1e-2 relative agreement, top-1 mostly equal)."""
import pytest
import torch

from anx.models.alexnet_full import FLOPS_PER_IMAGE, AlexNetFull, init_full_weights, reference_forward, weight_shapes
from anx.utils.init import init_input


def test_weight_shapes_and_init():
    shapes, b = weight_shapes(1000)
    assert shapes[0] == (96, 3, 11, 11) and shapes[5] == (4096, 9216) and shapes[7] == (1000, 4096)
    w = init_full_weights(3)
    assert w["w_conv1"].shape == (96, 3, 11, 11) and w["b_fc8"].shape == (1000,)
    assert torch.equal(w["w_fc7"], init_full_weights(3)["w_fc7"])  # deterministic
    assert 2.2e9 < FLOPS_PER_IMAGE < 2.3e9  # ungrouped Conv2 (the reference's), 2.27 GFLOP/image


def test_reference_forward_cpu_shapes():
    w = init_full_weights(1, classes=10)
    y = reference_forward(init_input(2, "rand", seed=1), w)
    assert y.shape == (2, 10) and torch.isfinite(y).all()


@pytest.mark.gpu
@pytest.mark.parametrize("N,groups2", [(3, 1), (64, 1), (2, 2)])
def test_full_alexnet_vs_torch(cuda, N, groups2):
    m = AlexNetFull(seed=5, device=cuda, max_batch=N, groups2=groups2)
    x = init_input(N, "rand", seed=5) * 10  # U[0,1): image-like dynamic range
    y = m(x.to(cuda)).cpu().double()
    ref = reference_forward(x, m.weights, groups2=groups2).double()
    rel = (y - ref).norm() / ref.norm()
    assert rel < 3e-2, rel
    assert (y.argmax(1) == ref.argmax(1)).float().mean() >= 0.6


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [2, 3])
def test_bf16_lds_dma_kernel_matches_register_staged(cuda, mode):
    """The LDS-DMA ring kernel (128x128 vec8 layers: conv2-5 at this batch, FC6-8) sums the same
    products in the same order as the register-staged kernel: logits bit-identical."""
    N = 160
    x = (init_input(N, "rand", seed=6) * 10).to(cuda)
    ref = AlexNetFull(seed=6, device=cuda, max_batch=N, knobs={"bf16_glds": 0})(x).clone()
    got = AlexNetFull(seed=6, device=cuda, max_batch=N, knobs={"bf16_glds": mode})(x)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.gpu
def test_full_conv1_polyphase_matches_taps8(cuda, monkeypatch):
    """Conv1 as a 3x3/1 conv over the 48-channel polyphase image (default) against the direct
    11x11/4 taps8 gathers (ANX_FULL_CONV1=taps8): same products, other bf16 summation order."""
    N = 16
    x = (init_input(N, "rand", seed=8) * 10).to(cuda)
    monkeypatch.setenv("ANX_FULL_CONV1", "taps8")
    ref = AlexNetFull(seed=8, device=cuda, max_batch=N)(x).clone()
    monkeypatch.delenv("ANX_FULL_CONV1")
    got = AlexNetFull(seed=8, device=cuda, max_batch=N)(x)
    torch.cuda.synchronize()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel
    assert (got.argmax(1) == ref.argmax(1)).float().mean() >= 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("lrn", ["div_n", "raw"])
def test_bf16_pool_lrn_wave_kernel_bitwise(cuda, monkeypatch, lrn):
    """Pool2+LRN2 as one wave per pixel (bpermute neighbours, default) against the LDS-tile kernel
    (ANX_BF16_LRN_TILE=1): same maxima, same ascending sums -> logits bit-identical."""
    N = 24
    x = (init_input(N, "rand", seed=9) * 10).to(cuda)
    monkeypatch.setenv("ANX_BF16_LRN_TILE", "1")
    m = AlexNetFull(seed=9, device=cuda, max_batch=N, lrn_mode=lrn)
    ref = m(x).clone()
    monkeypatch.delenv("ANX_BF16_LRN_TILE")
    got = m(x)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
