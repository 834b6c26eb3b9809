"""Per-layer ops (anx.ops) against PyTorch fp64 references of the same op, and the P7 filter-parallel
strategy (anx.parallel.tensor): every shard count must reproduce the unsharded result bit for bit
(same ops, per-filter-independent Conv2, exact zero channel halo at the edges), on CPU ranks
over gloo and on the GPU."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import anx  # noqa: E402,F401
from anx import ops  # noqa: E402
from anx.config import BLOCK1, BLOCK2  # noqa: E402
from anx.models.reference import blocks_forward, lrn_nhwc  # noqa: E402
from anx.parallel import tensor as tp  # noqa: E402
from anx.utils.init import init_input, init_weights  # noqa: E402


def _ref_conv(x, w, b, s, p, g, relu):
    y = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), stride=s, padding=p, groups=g)
    y = y.permute(0, 2, 3, 1)
    return y.clamp(min=0) if relu else y


CONV_CASES = [  # N, H, C, K, F, S, P, groups
    (2, 23, 3, 16, 11, 4, 0, 1),   # conv1-like (taps4 gather on the GPU)
    (2, 13, 8, 12, 5, 1, 2, 1),
    (1, 9, 8, 8, 3, 1, 1, 2),
    (3, 7, 4, 32, 1, 1, 0, 1),     # 1x1
]


def _conv_case(device, case):
    N, H, C, K, Fk, S, P, g = case
    gen = torch.Generator().manual_seed(sum(case))
    x = torch.rand(N, H, H, C, generator=gen)
    w = torch.rand(K, C // g, Fk, Fk, generator=gen) - 0.5
    b = torch.rand(K, generator=gen)
    y = ops.conv2d(x.to(device), w, b, S, P, g, relu=True).cpu()
    ref = _ref_conv(x, w, b, S, P, g, True)
    torch.testing.assert_close(y.double(), ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_cpu(case):
    _conv_case("cpu", case)


def test_pool_lrn_cpu():
    x = torch.rand(2, 9, 9, 12)
    p = ops.maxpool(x, 3, 2)
    torch.testing.assert_close(p, F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2).permute(0, 2, 3, 1))
    for mode in ("div_n", "raw"):
        y = ops.lrn(p.contiguous(), 5, 1e-4, 0.75, 2.0, mode)
        torch.testing.assert_close(y.double(), lrn_nhwc(p.double(), 5, 1e-4, 0.75, 2.0, mode), rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(ops.maxpool_lrn(x, mode=mode), ops.lrn(p.contiguous(), mode=mode))


def test_filter_ranges():
    for K in (5, 256, 257):
        for ws in range(1, 9):
            r = tp.filter_ranges(K, ws)
            assert r[0].lo == 0 and r[-1].hi == K and all(a.hi == b.lo for a, b in zip(r, r[1:]))
            assert max(x.size for x in r) - min(x.size for x in r) <= 1


@pytest.fixture(scope="module")
def small_case():
    return init_input(1, "rand", seed=4), init_weights("rand", 4)


@pytest.mark.parametrize("ws", [2, 3, 8])
def test_filter_shards_bitwise_cpu(small_case, ws):
    x, w = small_case
    full = tp.simulate(x, w, 1)
    torch.testing.assert_close(tp.simulate(x, w, ws), full, rtol=0, atol=0)
    ref = blocks_forward(x, w, BLOCK1, BLOCK2)
    torch.testing.assert_close(full.double(), ref, rtol=2e-5, atol=1e-3)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tp_worker(rank, ws, port, q):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.parallel import tensor as tp_
    from anx.utils.init import init_input as ii, init_weights as iw
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    torch.set_num_threads(1)
    y = tp_.filter_parallel_forward(ii(1, "rand", seed=4), iw("rand", 4), gather="all")
    yr = tp_.filter_parallel_forward(ii(1, "rand", seed=4), iw("rand", 4), gather="root")
    if rank == 0:
        q.put((y.clone(), yr.clone()))
    else:
        assert yr is None
    dist.barrier()
    dist.destroy_process_group()


def test_filter_parallel_gloo(small_case):
    ws = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    y, yr = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = tp.simulate(*small_case, 1)
    torch.testing.assert_close(y, full, rtol=0, atol=0)
    torch.testing.assert_close(yr, full, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_gpu(cuda, case):
    _conv_case(cuda, case)


@pytest.mark.gpu
def test_pool_lrn_gpu(cuda):
    x = torch.rand(2, 27, 27, 256)
    xg = x.to(cuda)
    p = ops.maxpool(xg, 3, 2)
    torch.testing.assert_close(p.cpu(), F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2).permute(0, 2, 3, 1))
    for mode in ("div_n", "raw"):
        ref = lrn_nhwc(p.cpu().double(), 5, 1e-4, 0.75, 2.0, mode)
        torch.testing.assert_close(ops.lrn(p, mode=mode).cpu().double(), ref, rtol=2e-6, atol=1e-6)
        torch.testing.assert_close(ops.maxpool_lrn(xg, mode=mode).cpu().double(), ref, rtol=2e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("ws", [2, 4, 8])
def test_filter_shards_bitwise_gpu(cuda, small_case, ws):
    x, w = small_case
    full = tp.simulate(x.to(cuda), w, 1)
    torch.testing.assert_close(tp.simulate(x.to(cuda), w, ws), full, rtol=0, atol=0)
    ref = blocks_forward(x, w, BLOCK1, BLOCK2)
    torch.testing.assert_close(full.cpu().double(), ref, rtol=2e-5, atol=1e-3)


@pytest.mark.gpu
def test_conv2d_weight_cache_not_fooled_by_address_reuse(cuda):
    """Two equal-shape temporary weight shards with different values, back to back (advisor round 1:
    the packed-weight cache was keyed by the data pointer without keeping the tensor alive, so the
    second shard could reuse the first's freed address and be served its filters). Each call must
    match its own fp64 reference; the first temporary is dropped before the second is made."""
    gen = torch.Generator().manual_seed(3)
    x = torch.rand(2, 13, 13, 8, generator=gen)
    full = torch.rand(16, 8, 5, 5, generator=gen) - 0.5
    b = torch.rand(8, generator=gen)
    outs = []
    for lo in (0, 8):
        shard = full[lo:lo + 8].contiguous()  # a fresh temporary of the same shape each time
        outs.append(ops.conv2d(x.to(cuda), shard, b, 1, 2, 1, relu=True).cpu())
        torch.testing.assert_close(outs[-1].double(), _ref_conv(x, shard, b, 1, 2, 1, True), rtol=2e-5, atol=2e-5)
        del shard
    assert not torch.equal(outs[0], outs[1])
