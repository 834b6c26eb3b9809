"""The native V5 runtime (csrc/src/runtime/v5.cpp, anx/v5.hpp) against its Python mirror, and on the GPU.

CPU: the runtime's record-only schedules (libanx_dist ``anx_v5_schedule``, no GPU) are exactly the
Python planner's :func:`anx.parallel.plan.step_schedule` (same transfers, same byte offsets, same
halo chunks, same order), every rank's transport issues precisely its share of that list, and the
balanced default decomposition stays within 10% of the mean work per rank.

GPU: ranks sharing the box's one GPU (peer transport, device-side flags or host notes) run the
pipelined, chunked schedule with every consumed buffer NaN-poisoned after use; the gathered output
must equal the single-GPU engine's. The native V4 runtime (anx/v4.hpp) likewise.
"""
import os
import socket
import sys
from collections import Counter

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from anx import _native as nat  # noqa: E402
from anx.parallel.plan import (OVERLAP, PER_LAYER, balanced_row_ways, make_hybrid_plan, plan_stats,  # noqa: E402
                               step_schedule)

pytestmark = pytest.mark.skipif(not os.path.exists(nat.DIST_PATH), reason="libanx_dist not built")

CASES = [(1, 4, -1), (2, 2, -1), (2, 3, 2), (3, 1, 3), (4, 8, -1), (4, 3, 0), (4, 5, 4), (8, 1024, -1), (8, 16, 8),
         (8, 2, -1), (8, 8, 1), (6, 7, 3), (8, 1024, 4)]


def _native(np_, batch, rw, layer=PER_LAYER, chunks=0, rank=-1, transport="rccl"):
    from anx.parallel.workloads import native_schedule
    return native_schedule(np_, batch, rw, layer, chunks, rank, transport)


@pytest.mark.parametrize("np_,batch,rw", CASES)
@pytest.mark.parametrize("layer,chunks", [(PER_LAYER, 0), (PER_LAYER, 3), (OVERLAP, 0)])
def test_native_schedule_is_the_python_schedule(np_, batch, rw, layer, chunks):
    r = balanced_row_ways(np_, batch) if rw < 0 else rw
    hp = make_hybrid_plan(227, 227, np_, batch, r, layer)
    py = step_schedule(hp, chunks)
    assert _native(np_, batch, rw, layer, chunks) == py
    assert any(l.startswith("scatter") for l in py) and any(l.startswith("gather") for l in py)
    halo = [l for l in py if l.startswith("halo_p1")]
    assert bool(halo) == (layer == PER_LAYER and max(hp.group_size) > 1)


@pytest.mark.parametrize("np_,batch,rw", [(2, 3, -1), (4, 8, -1), (4, 3, 4), (8, 64, -1), (3, 2, 3)])
@pytest.mark.parametrize("transport", ["rccl", "peer"])
def test_each_rank_issues_its_share(np_, batch, rw, transport):
    """Every transfer of the step is issued by exactly its two endpoints (once by the root for its own
    local copies), by both transports."""
    full = _native(np_, batch, rw)
    issued = Counter()
    for rank in range(np_):
        mine = _native(np_, batch, rw, rank=rank, transport=transport)
        assert set(mine) <= set(full)
        for l in mine:
            s, d = l.split(" ")[1].split("->")
            assert rank in (int(s), int(d))
        issued.update(mine)
    for l in full:
        s, d = l.split(" ")[1].split("->")
        assert issued[l] == (1 if s == d else 2), l
    assert Counter(sum((_native(np_, batch, rw, rank=q, transport="rccl") for q in range(np_)), [])) == \
        Counter(sum((_native(np_, batch, rw, rank=q, transport="peer") for q in range(np_)), []))


def test_balanced_default():
    """The default decomposition keeps the row split (a halo path) but balances it: 8 ranks x 1024
    images -> 4 groups of 2 ranks, max / mean work 1.077 (the 8-way split: 1.23) and a tenth of its
    redundant conv1 rows."""
    assert balanced_row_ways(8, 1024) == 2 and balanced_row_ways(2, 1024) == 2 and balanced_row_ways(1, 5) == 1
    st = plan_stats(make_hybrid_plan(227, 227, 8, 1024, 2, PER_LAYER))
    rows8 = plan_stats(make_hybrid_plan(227, 227, 8, 1024, 8, PER_LAYER))
    assert st["imbalance"] <= 1.1 < rows8["imbalance"]
    assert st["conv1_redundancy"] < rows8["conv1_redundancy"] / 4
    assert st["out_rows_max"] == 7 and abs(st["out_rows_mean"] - 6.5) < 1e-9
    for np_ in (2, 4, 8):
        for batch in (np_, 64, 1024):
            assert plan_stats(make_hybrid_plan(227, 227, np_, batch, balanced_row_ways(np_, batch),
                                               PER_LAYER))["imbalance"] <= 1.1


def test_chunks_cover_the_halo_images():
    """The halo chunks of a transfer tile its images exactly (no image sent twice or skipped)."""
    full = step_schedule(make_hybrid_plan(227, 227, 4, 10, 2, PER_LAYER), 3)
    halos = [l for l in full if l.startswith("halo_p1")]
    assert {l.split(" ")[0] for l in halos} == {"halo_p1#0", "halo_p1#1", "halo_p1#2"}
    per_edge = Counter()
    for l in halos:
        f = dict(kv.split("=") for kv in l.split(" ")[2:4])
        per_edge[l.split(" ")[1]] += int(f["h"])
    assert set(per_edge.values()) == {5}  # 10 images over 2 groups: every edge carries its group's 5


# ------------------------------------------------------------------------------------------ GPU
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _v5_rank(rank, world, port, q, kw, batch, steps, kind="v5"):
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
    sys.path.insert(0, ROOT)
    import torch as T
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.parallel.workloads import NativeV4, NativeV5
    from anx.utils.init import init_input
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        T.cuda.set_device(0)
        w = AlexNetBlocks(init="rand", seed=9, device="cpu", lrn_mode="raw").weights if rank == 0 else None
        from anx.config import blocks
        wl = (NativeV5 if kind == "v5" else NativeV4)(batch, w, specs=blocks("raw", 1), port=port, timeout_s=60, **kw)
        wl.fill(init_input(batch, "rand", seed=9) if rank == 0 else None)
        wl.step(steps=steps)
        wl.sync()
        # numpy, not a torch tensor: torch would share its storage through a file descriptor that
        # dies with this process
        out = (wl.output().numpy(), wl.describe(), wl.phase_ms()) if rank == 0 else None
        wl.close()
        q.put((rank, out))
    except Exception as e:  # pragma: no cover - reported by the parent
        q.put((rank, repr(e)))


def _run_v5(world, kw, batch=6, steps=4, kind="v5"):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_v5_rank, args=(r, world, port, q, kw, batch, steps, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not isinstance(v, str), f"rank {r}: {v}"
    return res[0]


@pytest.fixture(scope="module")
def v5_reference(cuda):
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    m = AlexNetBlocks(init="rand", seed=9, device="cuda", lrn_mode="raw", max_batch=6)
    y = m(init_input(6, "rand", seed=9).cuda()).cpu()
    m.close()
    return y


@pytest.mark.gpu
@pytest.mark.parametrize("world,kw", [
    (2, {"transport": "peer", "pipeline": 1, "poison": True}),
    (4, {"transport": "peer", "pipeline": 1, "poison": True, "chunks": 3}),
    (4, {"transport": "peer", "pipeline": 0, "poison": True, "decomp": "rows"}),
    (4, {"transport": "peer", "pipeline": 1, "poison": True, "peer_sync": "notes"}),
    (3, {"transport": "peer", "pipeline": 1, "poison": True, "layer": "overlap", "decomp": "rows"}),
    (1, {"pipeline": 1, "poison": True}),
])
def test_native_v5_shared_gpu(v5_reference, world, kw):
    """Pipelined chunked V5 through the C ABI (the bench's path) with NaN-poisoned buffers: equal to
    the single-GPU engine to fp32 rounding (Winograd tile origins move with the row split)."""
    y, desc, phases = _run_v5(world, kw)
    y = torch.from_numpy(y)
    err = (y - v5_reference).abs().max().item() / v5_reference.abs().max().item()
    assert err < 1e-5, (err, desc)
    assert desc["transport"] == kw.get("transport", "rccl" if world == 1 else "peer")
    assert set(phases) == {"scatter", "stage1", "halo_p1", "stage2", "gather"}
    if kw.get("transport") == "peer":
        assert desc["ordering"] == kw.get("peer_sync", "flags")


@pytest.mark.gpu
@pytest.mark.parametrize("world,kw", [(1, {}), (2, {}), (3, {"decomp": "rows", "chunks": 2}), (4, {"decomp": "hybrid"})])
def test_native_v4_shared_gpu(v5_reference, world, kw):
    """V4 through the native host-staged runtime (shared pinned segment, per-rank chunked H2D / tile /
    D2H on three streams, parity buffers across steps) on ranks sharing the GPU."""
    y, desc, phases = _run_v5(world, kw, kind="v4")
    y = torch.from_numpy(y)
    err = (y - v5_reference).abs().max().item() / v5_reference.abs().max().item()
    assert err < 1e-5, (err, desc)
    assert set(phases) == {"h2d", "compute", "d2h"} and phases["h2d"] > 0
    assert desc["runtime"].startswith("native") and desc["h2d_bytes_per_step_rank"] > 0
