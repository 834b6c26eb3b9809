"""GPU numerics: every native HIP kernel and engine path vs a plain PyTorch reference of the same
op (fp64 oracle), plus golden values and row-tile/halo decompositions on the device."""
import ctypes as C

import pytest
import torch

from anx import _native as nat
from anx.models.alexnet_blocks import AlexNetBlocks
from anx.models.reference import blocks_forward, blocks_forward_all, conv2d_nhwc, lrn_nhwc, maxpool_nhwc
from anx.parallel.plan import OVERLAP, PER_LAYER, make_plan
from anx.utils.init import init_input

pytestmark = pytest.mark.gpu

# Logged by the reference (its fp32 serial sums); BASELINE.md §4 notes the fp64 recomputation is
# 44.4147 42.4608 40.6963 — the log itself is 5e-4 off. Kernels that sum in a different order (MFMA
# tiles, Winograd) land on the fp64 value, so the logs are checked to 1e-3 and fp64 to 2e-4.
GOLD_DIV_N = [44.4152, 42.4612, 40.6967, 40.6967, 40.6967]
GOLD_DIV_N_F64 = [44.4147, 42.4608, 40.6963, 40.6963, 40.6963]
GOLD_RAW = [29.2932, 25.9153, 23.3255, 23.3255, 23.3255]


def test_native_library_loaded(cuda):
    assert nat.lib().anx_device_count() >= 1


@pytest.mark.parametrize("impl", ["mfma", "direct"])
@pytest.mark.parametrize("mode,gold", [("div_n", GOLD_DIV_N), ("raw", GOLD_RAW)])
def test_golden(cuda, impl, mode, gold):
    m = AlexNetBlocks(device=cuda, lrn_mode=mode, impl=impl)
    y = m(init_input(1, "const").to(cuda)).cpu()
    assert y.flatten()[:5].tolist() == pytest.approx(gold, abs=1e-3)
    if mode == "div_n":
        assert y.flatten()[:5].tolist() == pytest.approx(GOLD_DIV_N_F64, rel=2e-5)


@pytest.mark.parametrize("impl", ["mfma", "direct"])
@pytest.mark.parametrize("N", [1, 3, 64])
def test_engine_vs_oracle(cuda, impl, N):
    m = AlexNetBlocks(device=cuda, init="rand", seed=21, impl=impl, max_batch=N)
    x = init_input(N, "rand", seed=21)
    y = m(x.to(cuda)).cpu().double()
    ref = blocks_forward(x, m.weights, m.b1, m.b2)
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


def test_engine_grouped_conv2(cuda):
    m = AlexNetBlocks(device=cuda, init="rand", seed=4, groups2=2, max_batch=2)
    x = init_input(2, "rand", seed=4)
    torch.testing.assert_close(m(x.to(cuda)).cpu().double(), blocks_forward(x, m.weights, m.b1, m.b2),
                               rtol=2e-5, atol=2e-6)


def test_engine_large_batch_variant(cuda):
    """batch 256 runs the Winograd path in one launch per conv (both fused Winograd GEMMs at their
    largest grids, the band transforms, pool1 fused into the Conv2 input transform)."""
    N = 256
    m = AlexNetBlocks(device=cuda, init="rand", seed=8, max_batch=N)
    x = init_input(N, "rand", seed=8)
    y = m(x.to(cuda)).cpu()
    ref = blocks_forward_all(x, m.weights, m.b1, m.b2, device=cuda)  # every image, fp64
    torch.testing.assert_close(y.double(), ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("np_", [2, 4, 8])
def test_device_tiles(cuda, np_):
    m = AlexNetBlocks(device=cuda, init="rand", seed=9, max_batch=4)
    x = init_input(4, "rand", seed=9).to(cuda)
    full = m(x)
    p = make_plan(227, 227, np_, OVERLAP)
    parts = [m.tile_forward(x[:, t.inp.lo:t.inp.hi].contiguous(), t) for t in p.tiles if not t.out.empty]
    torch.testing.assert_close(torch.cat(parts, dim=1), full, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("np_", [2, 4, 8])
def test_device_per_layer_halo(cuda, np_):
    m = AlexNetBlocks(device=cuda, init="rand", seed=10, max_batch=2)
    x = init_input(2, "rand", seed=10).to(cuda)
    full = m(x)
    p = make_plan(227, 227, np_, PER_LAYER)
    engines = [AlexNetBlocks(device=cuda, weights=m.weights, max_batch=2) for _ in range(np_)]
    for r, t in enumerate(p.tiles):
        if not t.out.empty:
            engines[r].stage1(x[:, t.inp.lo:t.inp.hi].contiguous(), t)
    for h in p.p1_halos:
        engines[h.dst].window_put(p.tiles[h.dst], h.rows.lo,
                                  engines[h.src].window_get(p.tiles[h.src], h.rows.lo, h.rows.hi, 2))
    parts = [engines[r].stage2(2, t) for r, t in enumerate(p.tiles) if not t.out.empty]
    torch.testing.assert_close(torch.cat(parts, dim=1), full, rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------- single kernels
def _conv_mfma(x, w, b, S, P, groups, relu, out=None):
    """Run the native MFMA conv through the C ABI (pads on the host side of the contract)."""
    N, H, W, Cin = x.shape
    K = w.shape[0]
    xp = torch.nn.functional.pad(x, (0, 0, P, P, P, P)).contiguous()
    plan = (C.c_int * 16)()
    npk, nko = C.c_size_t(), C.c_size_t()
    nat.call("anx_conv_plan", N, H + 2 * P, W + 2 * P, Cin, K, w.shape[2], S, groups, plan, C.byref(npk),
             C.byref(nko))
    packed = torch.empty(npk.value)
    koff = torch.empty(nko.value, dtype=torch.int32)
    wc = w.detach().cpu().contiguous()
    nat.call("anx_conv_pack", plan, wc.data_ptr(), packed.data_ptr(), koff.data_ptr())
    packed, koff = packed.to(x.device), koff.to(x.device)
    Ho, Wo = plan[8], plan[9]
    y = torch.empty(N, Ho, Wo, K, device=x.device)
    nat.call("anx_conv2d_mfma", plan, xp.data_ptr(), packed.data_ptr(), koff.data_ptr(), b.data_ptr(), y.data_ptr(),
             Ho, Wo, K, 0, 0, 0, int(relu), nat.stream_ptr(x.device))
    return y


@pytest.mark.parametrize("shape", [
    # N, H, W, C, K, F, S, P, groups
    (1, 227, 227, 3, 96, 11, 4, 0, 1),
    (2, 27, 27, 96, 256, 5, 1, 2, 1),
    (2, 27, 27, 96, 256, 5, 1, 2, 2),
    (1, 13, 13, 256, 384, 3, 1, 1, 1),
    (3, 13, 13, 384, 256, 3, 1, 1, 2),
    (1, 9, 11, 5, 40, 3, 2, 1, 1),     # ragged: C%4!=0, K not a tile multiple
    (64, 27, 27, 96, 256, 5, 1, 2, 1),  # large-tile variant
])
def test_conv_mfma_vs_torch(cuda, shape):
    N, H, W, Cin, K, F, S, P, g = shape
    torch.manual_seed(0)
    x = torch.randn(N, H, W, Cin, device=cuda)
    w = torch.randn(K, Cin // g, F, F, device=cuda) * 0.1
    b = torch.randn(K, device=cuda)
    y = _conv_mfma(x, w, b, S, P, g, relu=True)
    ref = conv2d_nhwc(x.double(), w.double(), b.double(), S, P, g, relu=True)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-4)


def test_conv_direct_vs_torch(cuda):
    torch.manual_seed(1)
    x = torch.randn(2, 20, 21, 6, device=cuda)
    w = torch.randn(8, 3, 5, 5, device=cuda)
    b = torch.randn(8, device=cuda)
    y = torch.empty(2, 10, 11, 8, device=cuda)
    nat.call("anx_conv2d_direct", x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), 2, 20, 21, 6, 8, 5, 2, 2, 2,
             0, nat.stream_ptr(cuda))
    torch.testing.assert_close(y.double(), conv2d_nhwc(x.double(), w.double(), b.double(), 2, 2, 2), rtol=1e-5,
                               atol=1e-4)


def test_relu(cuda):
    x = torch.randn(1001, device=cuda)
    ref = torch.relu(x)
    nat.call("anx_relu", x.data_ptr(), x.numel(), nat.stream_ptr(cuda))
    torch.testing.assert_close(x, ref, rtol=0, atol=0)


@pytest.mark.parametrize("vec", [True, False])
def test_maxpool(cuda, vec):
    x = torch.randn(3, 27, 26, 96, device=cuda)
    ref = maxpool_nhwc(x, 3, 2)
    y = torch.empty_like(ref)
    if vec:
        nat.call("anx_maxpool", x.data_ptr(), 3, 27, 26, 96, 3, 2, y.data_ptr(), 13, 12, 96, 0, 0, 0,
                 nat.stream_ptr(cuda))
    else:
        nat.call("anx_maxpool_direct", x.data_ptr(), y.data_ptr(), 3, 27, 26, 96, 3, 2, nat.stream_ptr(cuda))
    torch.testing.assert_close(y, ref, rtol=0, atol=0)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("C", [256, 128])  # 256: wave-per-pixel kernel; else the LDS-tile kernel
def test_lrn_and_fused_pool_lrn(cuda, mode, C):
    x = torch.rand(2, 27, 27, C, device=cuda) * 4
    pooled = maxpool_nhwc(x, 3, 2)
    ref = lrn_nhwc(pooled.double(), 5, 1e-4, 0.75, 2.0, "div_n" if mode == 0 else "raw")
    y = torch.empty_like(pooled)
    nat.call("anx_lrn_direct", pooled.data_ptr(), y.data_ptr(), 2, 13, 13, C, 5, 1e-4, 0.75, 2.0, mode,
             nat.stream_ptr(cuda))
    torch.testing.assert_close(y.double(), ref, rtol=1e-6, atol=1e-6)
    y2 = torch.empty_like(pooled)
    nat.call("anx_maxpool_lrn", x.data_ptr(), y2.data_ptr(), 2, 27, 27, C, 3, 2, 5, 1e-4, 0.75, 2.0, mode,
             nat.stream_ptr(cuda))
    torch.testing.assert_close(y2.double(), ref, rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------- Winograd F(3x3,5x5) conv2
WINO2 = {"conv2_algo": "winograd"}
WINO1 = {"conv1_algo": "winograd"}


@pytest.mark.parametrize("N", [1, 5, 64])
@pytest.mark.parametrize("groups2", [1, 2])
def test_winograd_engine_vs_oracle(cuda, N, groups2):
    m = AlexNetBlocks(device=cuda, init="rand", seed=31 + N, max_batch=N, groups2=groups2, knobs=WINO2)
    x = init_input(N, "rand", seed=31 + N)
    y = m(x.to(cuda)).cpu().double()
    ref = blocks_forward(x, m.weights, m.b1, m.b2)
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("np_", [2, 3, 4, 8])
def test_winograd_row_tiles_partial(cuda, np_):
    """Row tiles give conv2 heights that are not multiples of 3 (partial Winograd tiles)."""
    m = AlexNetBlocks(device=cuda, init="rand", seed=40, max_batch=2, knobs=WINO2)
    x = init_input(2, "rand", seed=40)
    ref = blocks_forward(x, m.weights, m.b1, m.b2)
    xd = x.to(cuda)
    p = make_plan(227, 227, np_, OVERLAP)
    parts = [m.tile_forward(xd[:, t.inp.lo:t.inp.hi].contiguous(), t) for t in p.tiles if not t.out.empty]
    torch.testing.assert_close(torch.cat(parts, dim=1).cpu().double(), ref, rtol=2e-5, atol=2e-6)


def test_winograd_golden(cuda):
    m = AlexNetBlocks(device=cuda, lrn_mode="raw", knobs=WINO2)
    y = m(init_input(1, "const").to(cuda)).cpu()
    assert y.flatten()[:5].tolist() == pytest.approx(GOLD_RAW, abs=2e-4)


# ---------------------------------------------------------------- polyphase Winograd F(3x3,3x3) conv1
@pytest.mark.parametrize("shape", [
    # N, Hin, W, K, F
    (1, 227, 227, 96, 11),
    (3, 59, 47, 32, 11),    # ragged right/bottom tiles
    (2, 40, 61, 64, 9),     # F=9: the 4th phase row/col of every tap is zero
    (130, 227, 227, 96, 11),  # > one 128-tile block row, XCD-ordered grid with empty slots
])
def test_conv1_wino_kernel_vs_torch(cuda, shape):
    N, H, W, K, F = shape
    torch.manual_seed(3)
    x = torch.rand(N, H, W, 3, device=cuda)
    w = (torch.rand(K, 3, F, F) - 0.5) * 0.1
    b = torch.randn(K, device=cuda)
    H1, W1 = (H - F) // 4 + 1, (W - F) // 4 + 1
    y = torch.full((N, H1, W1, K), float("nan"), device=cuda)
    nat.call("anx_conv1_wino", x.data_ptr(), N, H, W, w.contiguous().data_ptr(), K, F, b.data_ptr(), y.data_ptr(), 0,
             nat.stream_ptr(cuda))
    ref = conv2d_nhwc(x.double(), w.to(cuda).double(), b.double(), 4, 0)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("occ1,occ2", [(0, 0), (2, 1), (3, 1)])
def test_winograd_gemm_occupancy_caps_bitwise(cuda, occ1, occ2):
    """The Winograd GEMMs' workgroups-per-CU caps (conv1_occ / conv2_occ: LDS padding) change only
    where workgroups run, never what they compute: outputs are bit-identical to the uncapped run."""
    x = init_input(9, "rand", seed=5).to(cuda)
    m = AlexNetBlocks(device=cuda, init="rand", seed=5, max_batch=9, knobs={**WINO1, **WINO2})
    y = m(x).clone()
    m.set_knob("conv1_occ", occ1)
    m.set_knob("conv2_occ", occ2)
    assert m.get_knob("conv1_occ") == occ1 and m.get_knob("conv2_occ") == occ2
    assert torch.equal(m(x), y)
    ref = blocks_forward(x.cpu(), m.weights, m.b1, m.b2)
    torch.testing.assert_close(y.cpu().double(), ref, rtol=2e-5, atol=2e-6)


def test_knobs_are_per_engine(cuda):
    """Two models in one process run different kernels at the same time; unknown knobs and bad
    values are rejected without changing the engine."""
    x = init_input(12, "rand", seed=8).to(cuda)
    a = AlexNetBlocks(device=cuda, init="rand", seed=8, max_batch=12, knobs={"conv2_algo": "direct"})
    b = AlexNetBlocks(device=cuda, init="rand", seed=8, max_batch=12, knobs={"conv2_algo": "winograd"})
    assert a.get_knob("conv2_algo") == 1 and b.get_knob("conv2_algo") == 2
    ya, yb = a(x), b(x)
    assert not torch.equal(ya, yb)  # different summation orders
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        a.set_knob("no_such_knob", 1)
    with pytest.raises(nat.NativeError):
        a.set_knob("conv1_occ", 99)
    assert a.get_knob("conv1_occ") == 0


@pytest.mark.parametrize("N", [1, 7, 128])
def test_conv1_winograd_engine_vs_oracle(cuda, N):
    m = AlexNetBlocks(device=cuda, init="rand", seed=50 + N, max_batch=N, knobs=WINO1)
    x = init_input(N, "rand", seed=50 + N)
    y = m(x.to(cuda)).cpu().double()
    torch.testing.assert_close(y, blocks_forward_all(x, m.weights, m.b1, m.b2, device=cuda), rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("np_", [2, 3, 4, 8])
def test_conv1_winograd_row_tiles(cuda, np_):
    """Row tiles start conv1's 3x3 Winograd tiles at the tile's own first row (partial tiles)."""
    m = AlexNetBlocks(device=cuda, init="rand", seed=60, max_batch=2, knobs=WINO1)
    x = init_input(2, "rand", seed=60)
    ref = blocks_forward(x, m.weights, m.b1, m.b2)
    xd = x.to(cuda)
    p = make_plan(227, 227, np_, OVERLAP)
    parts = [m.tile_forward(xd[:, t.inp.lo:t.inp.hi].contiguous(), t) for t in p.tiles if not t.out.empty]
    torch.testing.assert_close(torch.cat(parts, dim=1).cpu().double(), ref, rtol=2e-5, atol=2e-6)


def test_conv1_direct_and_winograd_agree(cuda):
    m = AlexNetBlocks(device=cuda, init="rand", seed=70, max_batch=4)
    x = init_input(4, "rand", seed=70).to(cuda)
    m.set_knob("conv1_algo", "direct")
    yd = m(x).clone()
    m.set_knob("conv1_algo", "winograd")
    yw = m(x)
    torch.testing.assert_close(yw, yd, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode,gold", [("div_n", GOLD_DIV_N_F64), ("raw", GOLD_RAW)])
def test_conv1_winograd_golden(cuda, mode, gold):
    # both convs Winograd (batch 1 would otherwise run conv2 direct: Auto picks direct below 9
    # images, whose 2400-term fp32 chains sit 1e-5 off the fp64 golden values)
    m = AlexNetBlocks(device=cuda, lrn_mode=mode, knobs={**WINO1, **WINO2})
    y = m(init_input(1, "const").to(cuda)).cpu()
    assert y.flatten()[:5].tolist() == pytest.approx(gold, abs=2e-4)


@pytest.mark.parametrize("N,groups2", [(9, 1), (9, 2), (300, 1), (130, 2)])
def test_winograd_conv2_gemm_sizes(cuda, N, groups2):
    """The fused Conv2 GEMM (64-tile x 64-filter workgroups, XCD-ordered grid with empty slots) at
    ragged tile counts, both group counts (96 / 48 channels per group), against the fp64 oracle."""
    m = AlexNetBlocks(device=cuda, init="rand", seed=80 + N, max_batch=N, groups2=groups2, knobs=WINO2)
    x = init_input(N, "rand", seed=80 + N)
    y = m(x.to(cuda)).cpu().double()
    torch.testing.assert_close(y, blocks_forward_all(x, m.weights, m.b1, m.b2, device=cuda), rtol=2e-5, atol=2e-6)


def test_engine_batch_above_launch_chunk(cuda):
    """Above ~1239 images the engine splits a forward into launches whose buffers stay below 2^31
    bytes (the Winograd GEMMs address their operands through 32-bit buffer offsets)."""
    N = 1300
    m = AlexNetBlocks(device=cuda, init="rand", seed=44, max_batch=N)
    x = init_input(N, "rand", seed=44)
    y = m(x.to(cuda))
    ref = blocks_forward_all(x, m.weights, m.b1, m.b2, device=cuda)  # every image, both launches, fp64
    torch.testing.assert_close(y.cpu().double(), ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("lanes,N", [(2, 150), (3, 200), (2, 100)])
def test_stream_lanes_bit_identical(cuda, lanes, N):
    """lanes > 1 splits the batch over concurrent HIP streams (one engine each): every image's output
    is bit-identical to the one-lane forward (same kernels per image), eager and under graph capture;
    below lanes * LANE_MIN images the forward stays on one stream."""
    from anx.models.alexnet_blocks import LANE_MIN
    x = (init_input(N, "rand", seed=13)).to(cuda)
    one = AlexNetBlocks(device=cuda, init="rand", seed=13, max_batch=N)
    many = AlexNetBlocks(one.weights, device=cuda, max_batch=N, lanes=lanes)
    assert len(many._lanes) == lanes - 1
    ref = one(x).clone()
    y = torch.full_like(ref, float("nan"))
    many(x, out=y)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    # graph capture of the forked/joined lanes, replayed on fresh input
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        many(x, out=y)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        many(x, out=y)
    x.copy_(init_input(N, "rand", seed=14).to(cuda))
    y.fill_(float("nan"))
    g.replay()
    ref2 = one(x)
    torch.cuda.synchronize()
    assert torch.equal(y, ref2)
    assert N >= lanes * LANE_MIN or torch.equal(many(x), ref2)


@pytest.mark.parametrize("N", [128, 300])
def test_forward_async_lanes_bit_identical(cuda, N):
    """forward_async (the bench's dp step: free-running lanes, no per-call join, lanes started half a
    forward apart when idle) computes exactly the one-lane forward, over repeated calls on the same
    buffers, after a device synchronisation (fresh start again), with per-lane hooks in order."""
    x = init_input(N, "rand", seed=31).to(cuda)
    one = AlexNetBlocks(device=cuda, init="rand", seed=31, max_batch=N)
    many = AlexNetBlocks(one.weights, device=cuda, max_batch=N, lanes=2)
    ref = one(x).clone()
    y = torch.full_like(ref, float("nan"))
    seen = []
    for _ in range(5):
        many.forward_async(x, y, on_lane=lambda i, lo, hi: seen.append((i, lo, hi)),
                           pre_lane=lambda i, lo, hi: seen.append(("pre", i)))
    many.join()
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert seen[:4] == [("pre", 0), (0, 0, N // 2), ("pre", 1), (1, N // 2, N)] and len(seen) == 20
    y.fill_(float("nan"))
    many.forward_async(x, y)
    many.join()
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("N,chunk", [(9, 0), (64, 0), (130, 0), (40, 16)])
def test_fused_pool1_bitwise(cuda, N, chunk):
    """Pool1 fused into the Winograd input transform (knob fuse_pool1, the tile_forward default) is
    bit-identical to the pool1 kernel + window + input transform, chunked launches included."""
    x = init_input(N, "rand", seed=11).to(cuda)
    kn = {**WINO1, **WINO2, "chunk1": chunk}
    fused = AlexNetBlocks(device=cuda, init="rand", seed=11, max_batch=N, knobs={**kn, "fuse_pool1": 1})
    plain = AlexNetBlocks(device=cuda, init="rand", seed=11, max_batch=N, knobs={**kn, "fuse_pool1": 0})
    y = fused(x)
    assert torch.equal(y, plain(x))
    ref = blocks_forward_all(x, fused.weights, fused.b1, fused.b2, device=cuda)
    torch.testing.assert_close(y.cpu().double(), ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("N,sub1,sub2", [(64, 16, 0), (64, 0, 24), (40, 16, 16), (20, 9, 12)])
def test_sub_chunks_bitwise(cuda, N, sub1, sub2):
    """Conv1 / Conv2 in sub-chunks (knobs conv1_sub / conv2_sub: the V workspace rewritten in place per
    sub-chunk) give the same bits as whole launches."""
    x = init_input(N, "rand", seed=15).to(cuda)
    whole = AlexNetBlocks(device=cuda, init="rand", seed=15, max_batch=N)
    sub = AlexNetBlocks(device=cuda, init="rand", seed=15, max_batch=N, knobs={"conv1_sub": sub1, "conv2_sub": sub2})
    assert torch.equal(whole(x), sub(x))


def test_fused_pool1_refuses_other_pool_shapes(cuda):
    """The fused pool1 + input transform kernel walks 3x3 / stride-2 windows only. A block-1 pool of
    another shape (2x2 / 2 also gives 27x27 here, so the rest of the engine is unchanged) must take
    the unfused pool1 kernel + window path with fuse_pool1 on: both knob settings agree bitwise and
    match the fp64 oracle of that spec."""
    from dataclasses import replace
    from anx.config import PoolSpec, blocks
    b1, b2 = blocks()
    b1 = replace(b1, pool=PoolSpec(2, 2))
    N = 12
    x = init_input(N, "rand", seed=14)
    kn = {**WINO1, **WINO2}
    on = AlexNetBlocks(device=cuda, init="rand", seed=14, max_batch=N, specs=(b1, b2), knobs={**kn, "fuse_pool1": 1})
    off = AlexNetBlocks(device=cuda, init="rand", seed=14, max_batch=N, specs=(b1, b2), knobs={**kn, "fuse_pool1": 0})
    y = on(x.to(cuda))
    assert torch.equal(y, off(x.to(cuda)))
    ref = blocks_forward(x[[0, N - 1]], on.weights, b1, b2)
    torch.testing.assert_close(y[[0, N - 1]].cpu().double(), ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("np_", [2, 3, 5])
def test_fused_pool1_row_tiles_bitwise(cuda, np_):
    """Overlap row tiles compute every pool1 row of their conv2 window: fused and unfused agree bitwise."""
    xd = init_input(12, "rand", seed=12).to(cuda)
    fused = AlexNetBlocks(device=cuda, init="rand", seed=12, max_batch=12, knobs={**WINO1, **WINO2})
    plain = AlexNetBlocks(device=cuda, init="rand", seed=12, max_batch=12, knobs={**WINO1, **WINO2, "fuse_pool1": 0})
    for t in make_plan(227, 227, np_, OVERLAP).tiles:
        if t.out.empty:
            continue
        xt = xd[:, t.inp.lo:t.inp.hi].contiguous()
        assert torch.equal(fused.tile_forward(xt, t), plain.tile_forward(xt, t))


@pytest.mark.parametrize("N,np_,form", [(7, 1, 1), (64, 1, 1), (6, 3, 1), (6, 5, 1), (7, 1, 2), (6, 5, 2)])
def test_conv1_band_transform_bitwise(cuda, N, np_, form):
    """The band forms of the Conv1 polyphase input transform (knob conv1_band: 1 = 2 phase rows per
    workgroup; 2 = 4 phase rows x half the tile columns, the default) give the same V as the per-tile
    gather kernel: whole images and overlap row tiles agree bitwise."""
    xd = init_input(N, "rand", seed=13).to(cuda)
    band = AlexNetBlocks(device=cuda, init="rand", seed=13, max_batch=N, knobs={**WINO1, **WINO2, "conv1_band": form})
    gath = AlexNetBlocks(device=cuda, init="rand", seed=13, max_batch=N, knobs={**WINO1, **WINO2, "conv1_band": 0})
    for t in make_plan(227, 227, np_, OVERLAP).tiles:
        if t.out.empty:
            continue
        xt = xd[:, t.inp.lo:t.inp.hi].contiguous()
        assert torch.equal(band.tile_forward(xt, t), gath.tile_forward(xt, t))


@pytest.mark.parametrize("mode", [1])
@pytest.mark.parametrize("N", [9, 33, 64, 130])
def test_conv1_fused_kernel(cuda, N, mode):
    """Conv1 as one kernel (knob conv1_fused: the polyphase input transform built in LDS inside the
    Winograd GEMM, 32 tiles x 96 filters per workgroup, U through an LDS ring) against the two-kernel
    form and the fp64 oracle, including partial tile blocks (P not a multiple of 32)."""
    x = init_input(N, "rand", seed=16)
    fused = AlexNetBlocks(device=cuda, init="rand", seed=16, max_batch=N, knobs={**WINO1, **WINO2, "conv1_fused": mode})
    plain = AlexNetBlocks(device=cuda, init="rand", seed=16, max_batch=N, knobs={**WINO1, **WINO2, "conv1_fused": 0})
    y, y0 = fused(x.to(cuda)), plain(x.to(cuda))
    assert (y - y0).abs().max().item() <= 1e-5 * y0.abs().max().item()
    ref = blocks_forward_all(x, fused.weights, fused.b1, fused.b2, device=cuda)
    torch.testing.assert_close(y.cpu().double(), ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("mode", [1])
@pytest.mark.parametrize("np_", [2, 3, 5])
def test_conv1_fused_row_tiles(cuda, np_, mode):
    """Overlap row tiles (fewer input rows than the image: the kernel zero-fills past the tile's last
    row) through the one-kernel Conv1 agree with the two-kernel form."""
    xd = init_input(12, "rand", seed=17).to(cuda)
    fused = AlexNetBlocks(device=cuda, init="rand", seed=17, max_batch=12, knobs={**WINO1, **WINO2, "conv1_fused": mode})
    plain = AlexNetBlocks(device=cuda, init="rand", seed=17, max_batch=12, knobs={**WINO1, **WINO2, "conv1_fused": 0})
    for t in make_plan(227, 227, np_, OVERLAP).tiles:
        if t.out.empty:
            continue
        xt = xd[:, t.inp.lo:t.inp.hi].contiguous()
        a, b = fused.tile_forward(xt, t), plain.tile_forward(xt, t)
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item()


@pytest.mark.parametrize("N,kn", [(9, {}), (33, {}), (64, {}), (130, {}), (40, {"chunk1": 16}),
                                  (64, {"conv2_sub": 24}), (20, {"chunk1": 9, "conv2_sub": 4})])
def test_conv1_pool_epilogue_bitwise(cuda, N, kn):
    """pool1 in the one-kernel Conv1's epilogue (knob conv1_pool: the conv1 map never reaches HBM; windows
    straddling two workgroups' tile ranges merged from a side buffer by the Conv2 input transform) gives
    the same bits as Conv1 writing its map and the input transform pooling it: partial workgroups (P
    not a multiple of 32), chunked launches and Conv2 sub-chunks (their offset into the Conv1 launch's
    tile numbering) included; the whole output is checked against the fp64 oracle too."""
    x = init_input(N, "rand", seed=21).to(cuda)
    base = {**WINO1, **WINO2, **kn}
    on = AlexNetBlocks(device=cuda, init="rand", seed=21, max_batch=N, knobs={**base, "conv1_pool": 1})
    off = AlexNetBlocks(device=cuda, init="rand", seed=21, max_batch=N, knobs={**base, "conv1_pool": 0})
    y = on(x)
    assert torch.equal(y, off(x))
    y.fill_(float("nan"))  # every pooled pixel rewritten each call (the window border stays zero)
    on(x, out=y)
    assert torch.equal(y, off(x))
    ref = blocks_forward(x.cpu(), on.weights, on.b1, on.b2)
    torch.testing.assert_close(y.cpu().double(), ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("N,kn,hw,mode", [(1, {}, None, "div_n"), (9, {}, None, "div_n"), (33, {}, None, "raw"),
                                          (64, {}, None, "div_n"), (130, {}, None, "div_n"),
                                          (40, {"chunk1": 16}, None, "div_n"), (64, {"conv2_sub": 24}, None, "div_n"),
                                          (20, {"chunk1": 9, "conv2_sub": 4}, None, "raw"),
                                          (5, {}, (195, 259), "div_n")])
def test_conv2_pool_epilogue_bitwise(cuda, N, kn, hw, mode):
    """pool2 in the F(4x4,5x5) Conv2 GEMM's epilogue (tuning knob conv2_pool: the conv2 map never reaches HBM;
    windows straddling two workgroups' 32-tile ranges merged from a side buffer by the LRN kernel) gives
    the same bits as the GEMM writing its map and maxpool_lrn pooling it: partial workgroups, chunks,
    Conv2 sub-chunks (the merge's image index inside a GEMM launch), both LRN modes and a non-square
    image; the whole output against the fp64 oracle too."""
    H, W = hw if hw else (227, 227)
    x = init_input(N, "rand", seed=23, H=H, W=W).to(cuda)
    base = {**WINO1, **WINO2, **kn}
    mk = lambda p: AlexNetBlocks(device=cuda, init="rand", seed=23, max_batch=N, H=H, W=W, lrn_mode=mode,
                                 knobs={**base, "conv2_pool": p})
    on, off = mk(1), mk(0)
    assert on.get_knob("conv2_pool") == 1 and off.get_knob("conv2_pool") == 0
    y = on(x)
    assert torch.equal(y, off(x))
    y.fill_(float("nan"))  # every pooled pixel rewritten each call
    on(x, out=y)
    assert torch.equal(y, off(x))
    ref = blocks_forward_all(x, on.weights, on.b1, on.b2, device=cuda)
    torch.testing.assert_close(y.double(), ref.to(cuda), rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("N,kn", [(9, {}), (64, {}), (130, {}), (300, {}), (40, {"chunk1": 16, "conv2_sub": 24})])
def test_conv2_hand_schedule_bitwise(cuda, N, kn):
    """The F(4x4,5x5) Conv2 GEMM's hand-scheduled K slice (knob conv2_sched = 1, wino_gemm16_sched.inc: counted
    fragment reads two groups ahead, the fold as a packed burst) gives the same bits as the compiler-scheduled
    kernel (same fmaf order per accumulator and fold value), on partial workgroups, multi-round grids and
    sub-chunked launches; the whole output against the fp64 oracle too."""
    x = init_input(N, "rand", seed=29).to(cuda)
    mk = lambda v: AlexNetBlocks(device=cuda, init="rand", seed=29, max_batch=N,
                                 knobs={**WINO1, **WINO2, **kn, "conv2_tile": 4, "conv2_sched": v})
    hand, comp = mk(1), mk(0)
    assert hand.get_knob("conv2_sched") == 1 and comp.get_knob("conv2_sched") == 0
    y = hand(x)
    assert torch.equal(y, comp(x))
    ref = blocks_forward_all(x, hand.weights, hand.b1, hand.b2, device=cuda)
    torch.testing.assert_close(y.double(), ref.to(cuda), rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("N", [9, 64, 130])
def test_lrn_grid_cap_bitwise(cuda, N):
    """The pool2-merge + LRN kernel with its grid capped (knob lrn_wgs: waves walk several pixel pairs) gives
    the same bits as one wave per pixel pair (lrn_wgs = 0), behind the pooled F(4x4,5x5) GEMM."""
    x = init_input(N, "rand", seed=31).to(cuda)
    mk = lambda v: AlexNetBlocks(device=cuda, init="rand", seed=31, max_batch=N,
                                 knobs={**WINO1, **WINO2, "conv2_tile": 4, "conv2_pool": 1, "lrn_wgs": v})
    capped, full, tiny = mk(256), mk(0), mk(3)
    assert capped.get_knob("lrn_wgs") == 256 and full.get_knob("lrn_wgs") == 0
    y = capped(x)
    assert torch.equal(y, full(x)) and torch.equal(y, tiny(x))


def test_set_knob_rebuilds_conv2_workspace(cuda):
    """conv2_tile switched 4 -> 3 -> 4 on one engine between forwards rebuilds the transformed weights and
    the V workspace each time (BlocksEngine::prepare) and matches engines built fresh with that tile
    (set_knob frees buffers a captured graph would still name, so it is a between-forwards
    operation)."""
    N = 24
    x = init_input(N, "rand", seed=31).to(cuda)
    fresh = {t: AlexNetBlocks(device=cuda, init="rand", seed=31, max_batch=N, knobs={**WINO2, "conv2_tile": t})(x)
             for t in (3, 4)}
    m = AlexNetBlocks(device=cuda, init="rand", seed=31, max_batch=N, knobs={**WINO2, "conv2_tile": 4})
    for t in (4, 3, 4, 3):
        m.set_knob("conv2_tile", t)
        assert m.get_knob("conv2_tile") == t
        assert torch.equal(m(x), fresh[t])


@pytest.mark.parametrize("um", [2, 3])
@pytest.mark.parametrize("N,kn", [(9, {}), (33, {}), (64, {}), (130, {}), (40, {"chunk1": 16})])
def test_conv1_per_wave_u_ring_bitwise(cuda, N, kn, um):
    """The one-kernel Conv1 with a private U ring per wave (knob conv1_fused = 2: each wave DMAs the filter
    rows its own fragments read and waits for them with its own vmcnt; barriers only where V is published) or
    with U in registers (3: each wave loads its B fragments from L2 one point ahead) gives the same bits as the
    shared-ring kernel (same MFMA and fold order), partial workgroups and chunked launches included; the whole
    output against the fp64 oracle too."""
    x = init_input(N, "rand", seed=37).to(cuda)
    base = {**WINO1, **WINO2, **kn, "conv1_pool": 1}
    upw = AlexNetBlocks(device=cuda, init="rand", seed=37, max_batch=N, knobs={**base, "conv1_fused": um})
    ring = AlexNetBlocks(device=cuda, init="rand", seed=37, max_batch=N, knobs={**base, "conv1_fused": 1})
    assert upw.get_knob("conv1_fused") == um
    y = upw(x)
    assert torch.equal(y, ring(x))
    ref = blocks_forward_all(x, upw.weights, upw.b1, upw.b2, device=cuda)
    torch.testing.assert_close(y.double(), ref.to(cuda), rtol=2e-5, atol=2e-6)
