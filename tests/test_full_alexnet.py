"""Full-AlexNet bf16 extension: shapes/init on the CPU; on the GPU every layer against a
bf16-quantising PyTorch oracle (same bf16 rounding points as the engine: inputs, weights and each
layer's stored output; fp64 math in between), plus end-to-end logits vs the fp32 oracle."""
import pytest
import torch
import torch.nn.functional as F

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


@pytest.mark.gpu
def test_full_alexnet_rejects_bad_buffers(cuda):
    """forward / forward_async write through raw pointers: a wrong x or out is refused, never written."""
    m = AlexNetFull(seed=5, device=cuda, max_batch=4, classes=10, lanes=2)
    x = init_input(4, "rand", seed=5).to(cuda)
    good = torch.empty(4, 10, device=cuda)
    bad = [torch.empty(4, 11, device=cuda), torch.empty(3, 10, device=cuda), torch.empty(4, 10),
           torch.empty(4, 10, device=cuda, dtype=torch.float16), torch.empty(10, 4, device=cuda).t()]
    for out in bad:
        for fn in (m.forward, m.forward_async):
            with pytest.raises(ValueError):
                fn(x, out)
    for xb in (x.cpu(), x[:, :, :200], x.half(), x.permute(0, 2, 1, 3)):
        with pytest.raises(ValueError):
            m.forward(xb, good)
    m.forward_async(x, good)
    m.join()
    torch.testing.assert_close(good, m(x), rtol=0, atol=0)
    m.close()


def _q(t):  # round to bf16, compute in fp64
    return t.to(torch.bfloat16).double()


@pytest.mark.gpu
def test_s2d4_polyphase_input_exact(cuda):
    """Conv1's polyphase input (tap 10): bf16(x) space-to-depth by 4, zero past the 227th row and
    column, [N, 57, 57, (rh*4 + rw)*3 + c] — bit-exact against the same rearrangement in torch (one
    round-to-nearest-even conversion on both sides)."""
    N = 5
    m = AlexNetFull(seed=3, device=cuda, max_batch=N, knobs={"bf16_conv1": 0})  # the s2d4 pass writes tap 10
    x = (torch.randn(N, 227, 227, 3, generator=torch.Generator().manual_seed(4)) * 3).to(cuda)
    m(x)
    xq = F.pad(x.to(torch.bfloat16), (0, 0, 0, 1, 0, 1))  # 228 x 228
    ref = xq.reshape(N, 57, 4, 57, 4, 3).permute(0, 1, 3, 2, 4, 5).reshape(N, 57, 57, 48)
    assert torch.equal(m.tap(10, N), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("groups2", [1, 2])
def test_full_alexnet_per_layer_vs_bf16_oracle(cuda, groups2):
    """Each layer of the engine, fed the engine's own (bf16) input of that layer, against the same
    layer in fp64 on bf16-rounded operands, rounded to bf16: only the fp32 summation order differs,
    so every layer agrees to <= 1e-2 of its max (|one bf16 ulp| = 0.4 %) and <= 4e-3 in L2."""
    N = 6
    m = AlexNetFull(seed=9, device=cuda, max_batch=N, groups2=groups2, knobs={"bf16_pool1": 0})  # conv1 map in tap 0
    x = (init_input(N, "rand", seed=9) * 10).to(cuda)
    logits = m(x).double()
    taps = [m.tap(i, N).double() for i in range(10)]
    w = {k: v.to(cuda) for k, v in m.weights.items()}
    nchw = lambda t: t.permute(0, 3, 1, 2)  # noqa: E731
    nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731

    def conv(h, name, stride=1, pad=0, groups=1, relu=True):
        y = F.conv2d(nchw(h), _q(w["w_" + name]), _q(w["b_" + name]), stride=stride, padding=pad, groups=groups)
        return nhwc(F.relu(y) if relu else y)

    def check(got, ref, what):
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        l2 = ((got - ref).norm() / ref.norm()).item()
        assert err <= 1e-2 and l2 <= 4e-3, (what, err, l2)

    pool = lambda h: nhwc(F.max_pool2d(nchw(h), 3, 2))  # noqa: E731
    check(taps[0], _q(conv(_q(x), "conv1", stride=4)), "conv1")
    check(taps[1][:, 2:-2, 2:-2], pool(taps[0]), "pool1")
    check(taps[2], _q(conv(taps[1], "conv2", groups=groups2)), "conv2")
    lrn = nhwc(F.local_response_norm(nchw(pool(taps[2])), 5, alpha=1e-4, beta=0.75, k=2.0))
    check(taps[3][:, 1:-1, 1:-1], _q(lrn), "pool2+lrn")
    check(taps[4][:, 1:-1, 1:-1], _q(conv(taps[3], "conv3")), "conv3")
    check(taps[5][:, 1:-1, 1:-1], _q(conv(taps[4], "conv4")), "conv4")
    check(taps[6], _q(conv(taps[5], "conv5")), "conv5")
    check(taps[7], pool(taps[6]).reshape(N, -1), "pool5")
    fc = lambda h, k, relu=True: (F.relu if relu else (lambda t: t))(  # noqa: E731
        h @ _q(w["w_" + k]).T + _q(w["b_" + k]))
    check(taps[8], _q(fc(taps[7], "fc6")), "fc6")
    check(taps[9], _q(fc(taps[8], "fc7")), "fc7")
    check(logits, fc(taps[9], "fc8", relu=False), "fc8")
    # the borders of the padded windows stay zero
    assert taps[1][:, :2].abs().max() == 0 and taps[3][:, :, :1].abs().max() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [2, 3])
def test_bf16_lds_dma_kernel_matches_register_staged(cuda, mode):
    """The LDS-DMA ring kernel (128x128 vec8 layers: conv2-5 at this batch, FC6-8) sums the same
    products in the same order as the register-staged kernel: logits bit-identical."""
    N = 160
    x = (init_input(N, "rand", seed=6) * 10).to(cuda)
    ref = AlexNetFull(seed=6, device=cuda, max_batch=N, knobs={"bf16_glds": 0, "bf16_big": -2})(x).clone()
    got = AlexNetFull(seed=6, device=cuda, max_batch=N, knobs={"bf16_glds": mode, "bf16_big": -2})(x)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [-1, 0, 1, 2, 3, 4, 12, 13, 14, 15, 16])
def test_bf16_wide_tile_kernel_matches_register_staged(cuda, cfg):
    """The wide-tile kernel (conv_bf16_big.hip; -1 = the cost model's per-layer pick, else that
    config forced wherever it fits) sums each output's products in the register-staged kernel's
    order: conv1..pool5 activations bit-identical. FC6-8 run K split another number of ways, so
    they agree to summation order only."""
    N = 37  # partial M tiles everywhere
    x = (init_input(N, "rand", seed=12) * 10).to(cuda)
    ref_m = AlexNetFull(seed=12, device=cuda, max_batch=N, knobs={"bf16_glds": 0, "bf16_big": -2})
    ref = ref_m(x).double()
    ref_taps = [ref_m.tap(i, N) for i in range(10)]
    m = AlexNetFull(seed=12, device=cuda, max_batch=N, knobs={"bf16_big": cfg})
    got = m(x).double()
    for i in range(8):
        assert torch.equal(m.tap(i, N), ref_taps[i]), i
    for i in (8, 9):
        t, r = m.tap(i, N).double(), ref_taps[i].double()
        assert ((t - r).norm() / r.norm()).item() < 1e-2, i
    assert ((got - ref).norm() / ref.norm()).item() < 1e-2


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
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("N", [1, 3, 40, 300])
def test_conv1_ring_kernel_matches_tile_kernels(cuda, N, mode):
    """Conv1 as the persistent row-band kernel (knob bf16_conv1=1: polyphase rows in an LDS ring,
    weights resident, 32x32x16 MFMA; 2: the same reading the fp32 image, space-to-depth + bf16
    inside) against s2d4 + the implicit-GEMM tile kernels (bf16_conv1=0): the same bf16 products in
    another fp32 summation order, so conv1 outputs agree to about one bf16 ulp; the segment split
    (N < CUs: an image's 14 row tiles over several workgroups) and the one-image-per-workgroup form
    are both covered."""
    x = (torch.randn(N, 227, 227, 3, generator=torch.Generator().manual_seed(N)) * 3).to(cuda)
    m = AlexNetFull(seed=19, device=cuda, max_batch=N, knobs={"bf16_conv1": mode, "bf16_pool1": 0})
    y = m(x).clone()
    c1 = m.tap(0, N).double()
    m.set_knob("bf16_conv1", 0)
    y0 = m(x)
    r1 = m.tap(0, N).double()
    torch.cuda.synchronize()
    assert (c1 - r1).abs().max().item() <= 1.6e-2 * r1.abs().max().item()
    assert ((c1 - r1).norm() / r1.norm()).item() < 4e-3
    assert ((y - y0).norm() / y0.norm()).item() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N", [256, 300, 40])
def test_conv1_ring_fused_pool1_exact(cuda, N):
    """pool1 in the ring kernel's epilogue (knob bf16_pool1=1; one workgroup per image from N = 256
    CUs on; below that the kernel writes the 55x55 map and maxpool_bf16 follows): the pooled map
    (tap 1, zero borders included) and the logits are bit-identical to Conv1 + the separate pool."""
    x = (torch.randn(N, 227, 227, 3, generator=torch.Generator().manual_seed(N + 1)) * 3).to(cuda)
    m = AlexNetFull(seed=31, device=cuda, max_batch=N, knobs={"bf16_pool1": 0})
    y0 = m(x).clone()
    q0 = m.tap(1, N).clone()
    m.set_knob("bf16_pool1", 1)
    y1 = m(x)
    q1 = m.tap(1, N)
    torch.cuda.synchronize()
    assert torch.equal(q1, q0)
    assert torch.equal(y1, y0)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [300, 512])
def test_full_lanes_pool1_paths_match_one_lane(cuda, N):
    """Two stream lanes (forward_async) split the batch: at 300 each lane's 150 images take the
    unfused Conv1 + maxpool fallback, at 512 each lane's 256 take pool1 inside the ring kernel — lane
    0's pooled map is bit-identical to the one-lane forward's first half either way, and the logits
    agree to the FC layers' split-K summation order."""
    x = (torch.randn(N, 227, 227, 3, generator=torch.Generator().manual_seed(N + 7)) * 3).to(cuda)
    one = AlexNetFull(seed=37, device=cuda, max_batch=N)
    ref = one(x).clone()
    ref_q = one.tap(1, N)[: N // 2].clone()
    m = AlexNetFull(seed=37, device=cuda, max_batch=N, lanes=2)
    out = torch.empty_like(ref)
    m.forward_async(x, out)
    m.join()
    torch.cuda.synchronize()
    assert torch.equal(m.tap(1, N // 2), ref_q)
    assert ((out.double() - ref.double()).norm() / ref.double().norm()).item() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [1, 2, 3])
def test_conv1_ring_fp32_input_interior_pointer(cuda, shift):
    """The fused-input ring (bf16_conv1=2) reads the fp32 image with aligned 16-B window loads from the
    granule holding x: an input that starts `shift` floats into a granule (a lane's x[lo:hi] slice or
    any interior view) gives the same Conv1 as an aligned copy, including the batch's last row, which
    takes the dword path."""
    N = 5
    flat = torch.randn(N * 227 * 227 * 3 + 8, generator=torch.Generator().manual_seed(shift)).to(cuda) * 3
    x = flat[shift:shift + N * 227 * 227 * 3].view(N, 227, 227, 3)
    assert (x.data_ptr() // 4) % 4 == shift % 4
    m = AlexNetFull(seed=29, device=cuda, max_batch=N, knobs={"bf16_conv1": 2})
    m(x)
    c_view = m.tap(0, N).clone()
    m(x.clone())
    c_copy = m.tap(0, N)
    torch.cuda.synchronize()
    assert torch.equal(c_view, c_copy)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 5])
def test_fc_forced_wide_tile_configs(cuda, cfg):
    """FC6-8 on a forced wide-tile config (knob bf16_fc_cfg, its own K split <= 16 slabs) against the
    default cfg 8: the same bf16 products summed in another order."""
    N = 40
    x = (init_input(N, "rand", seed=23) * 10).to(cuda)
    m = AlexNetFull(seed=23, device=cuda, max_batch=N)
    ref = m(x).clone()
    ref_taps = [m.tap(i, N).double() for i in (8, 9)]
    m.set_knob("bf16_fc_cfg", cfg)
    got = m(x)
    torch.cuda.synchronize()
    for i, r in zip((8, 9), ref_taps):
        t = m.tap(i, N).double()
        assert ((t - r).norm() / r.norm()).item() < 1e-2, i
    assert ((got - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("lrn", ["div_n", "raw"])
def test_bf16_pool_lrn_wave_kernel_bitwise(cuda, lrn):
    """Pool2+LRN2 as half-wave pixels (bpermute neighbours, default) against the LDS-tile kernel
    (knob bf16_lrn_tile=1): same maxima, same ascending sums -> logits bit-identical."""
    N = 25  # odd pixel count: the last wave step holds a lone pixel
    x = (init_input(N, "rand", seed=9) * 10).to(cuda)
    m = AlexNetFull(seed=9, device=cuda, max_batch=N, lrn_mode=lrn, knobs={"bf16_lrn_tile": 1})
    ref = m(x).clone()
    m.set_knob("bf16_lrn_tile", 0)
    got = m(x)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.gpu
def test_full_alexnet_lanes_bit_identical(cuda):
    """lanes=2 splits the batch over two engines on concurrent streams: every image's logits are
    bit-identical to the one-lane forward of the same images at that lane's batch size."""
    N = 10
    x = (init_input(N, "rand", seed=15) * 10).to(cuda)
    two = AlexNetFull(seed=15, device=cuda, max_batch=N, lanes=2)
    y = two(x).clone()
    one = AlexNetFull(two.weights, device=cuda, max_batch=N // 2)
    ref = torch.cat([one(x[:N // 2].contiguous()).clone(), one(x[N // 2:].contiguous()).clone()])
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.gpu
def test_full_alexnet_forward_async_bit_identical(cuda):
    """forward_async (free-running lanes, lane 1 started at lane 0's mid-forward mark when idle)
    equals the joined lane forward over repeated calls on the same buffers and after a device sync."""
    N = 10
    x = (init_input(N, "rand", seed=16) * 10).to(cuda)
    two = AlexNetFull(seed=16, device=cuda, max_batch=N, lanes=2)
    ref = two(x).clone()
    y = torch.full_like(ref, float("nan"))
    for _ in range(4):
        two.forward_async(x, y)
    two.join()
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    y.fill_(float("nan"))
    two.forward_async(x, y)
    two.join()
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
