"""The native V5 runtime (csrc/src/runtime/v5.cpp, anx/v5.hpp) against its Python mirror, and on the GPU.

CPU: the runtime's record-only schedules (libanx_dist ``anx_v5_schedule``, no GPU) are exactly the
Python planner's :func:`anx.parallel.plan.step_schedule` (same transfers, same byte offsets, same
halo chunks, same order; scatter only with root input), every rank's transport issues precisely its
share of that list, and the default decomposition is the cost model's pick.

GPU: ranks sharing the box's one GPU run the pipelined, chunked schedule with every consumed buffer
NaN-poisoned after use, over the peer transport (device-side flags or host notes) and over the RCCL
transport's own code on the loopback device comm (pack / staging / grouped P2P / unpack, two chained
communicators); the gathered output must equal the single-GPU engine's (bitwise with the direct
convolutions, which do not depend on tile origins), and the loopback run's transfer log must be the
record-only schedule. The native V4 runtime (anx/v4.hpp) likewise.
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
from anx.parallel.plan import (OVERLAP, PER_LAYER, make_hybrid_plan, pick_row_ways, plan_stats,  # noqa: E402
                               step_schedule)

pytestmark = pytest.mark.skipif(not os.path.exists(nat.DIST_PATH), reason="libanx_dist not built")

CASES = [(1, 4, -1), (2, 2, -1), (2, 3, 2), (3, 1, 3), (4, 8, -1), (4, 3, 0), (4, 5, 4), (8, 1024, -1), (8, 16, 8),
         (8, 2, -1), (8, 8, 1), (6, 7, 3), (8, 1024, 4)]


def _native(np_, batch, rw, layer=PER_LAYER, chunks=0, rank=-1, transport="rccl", src="root"):
    from anx.parallel.workloads import native_schedule
    return native_schedule(np_, batch, rw, layer, chunks, rank, transport, input_source=src)


@pytest.mark.parametrize("np_,batch,rw", CASES)
@pytest.mark.parametrize("layer,chunks", [(PER_LAYER, 0), (PER_LAYER, 3), (OVERLAP, 0)])
@pytest.mark.parametrize("src", ["root", "local"])
def test_native_schedule_is_the_python_schedule(np_, batch, rw, layer, chunks, src):
    r = pick_row_ways(np_, batch, "v5", src, layer) if rw < 0 else rw
    hp = make_hybrid_plan(227, 227, np_, batch, r, layer)
    py = step_schedule(hp, chunks, input_source=src)
    assert _native(np_, batch, rw, layer, chunks, src=src) == py
    assert any(l.startswith("scatter") for l in py) == (src == "root") and any(l.startswith("gather") for l in py)
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


def test_default_split_is_the_cost_model_pick():
    """The default decomposition is the cost model's (anx/cost.hpp): with local input the batch split
    (no halo, no redundant conv1, perfectly balanced) whenever every rank gets whole images. A forced
    2-way split stays balanced (8 x 1024: max / mean 1.077)."""
    assert pick_row_ways(8, 1024) == 1 and pick_row_ways(2, 1024) == 1 and pick_row_ways(1, 5) == 1
    st = plan_stats(make_hybrid_plan(227, 227, 8, 1024, 2, PER_LAYER))
    rows8 = plan_stats(make_hybrid_plan(227, 227, 8, 1024, 8, PER_LAYER))
    assert st["imbalance"] <= 1.1 < rows8["imbalance"]
    assert st["conv1_redundancy"] < rows8["conv1_redundancy"] / 4
    assert st["out_rows_max"] == 7 and abs(st["out_rows_mean"] - 6.5) < 1e-9
    assert plan_stats(make_hybrid_plan(227, 227, 8, 1024, 1, PER_LAYER))["imbalance"] == 1.0


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


def _v5_rank(rank, world, port, q, kw, batch, steps, kind="v5", env=None):
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
    os.environ.update(env or {})  # ANX_* knob seeds (before the engines are built)
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
        log = wl.transfer_log() if kw.get("keep_log") else None
        # numpy, not a torch tensor: torch would share its storage through a file descriptor that
        # dies with this process
        out = (wl.output().numpy(), wl.describe(), wl.phase_ms(), log) if rank == 0 else log
        wl.close()
        q.put((rank, out))
    except Exception as e:  # pragma: no cover - reported by the parent
        q.put((rank, repr(e)))


def _run_v5(world, kw, batch=6, steps=4, kind="v5", env=None, all_ranks=False):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_v5_rank, args=(r, world, port, q, kw, batch, steps, kind, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not isinstance(v, str), f"rank {r}: {v}"
    return res if all_ranks else res[0][:3]


def _reference(knobs=None, batch=6):
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    m = AlexNetBlocks(init="rand", seed=9, device="cuda", lrn_mode="raw", max_batch=batch, knobs=knobs or {})
    y = m(init_input(batch, "rand", seed=9).cuda()).cpu()
    m.close()
    return y


@pytest.fixture(scope="module")
def v5_reference(cuda):
    return _reference()


@pytest.fixture(scope="module")
def v5_reference_direct(cuda):
    return _reference({"conv1_algo": "direct", "conv2_algo": "direct"})


DIRECT_ENV = {"ANX_CONV1_ALGO": "direct", "ANX_CONV2_ALGO": "direct"}


@pytest.mark.gpu
@pytest.mark.parametrize("world,kw", [
    (2, {"transport": "peer", "pipeline": 1, "poison": True, "decomp": "rows"}),
    (4, {"transport": "peer", "pipeline": 1, "poison": True, "chunks": 3, "decomp": "rows"}),
    (4, {"transport": "peer", "pipeline": 0, "poison": True, "decomp": "rows", "input_source": "root"}),
    (4, {"transport": "peer", "pipeline": 1, "poison": True, "peer_sync": "notes", "decomp": "hybrid"}),
    (3, {"transport": "peer", "pipeline": 1, "poison": True, "layer": "overlap", "decomp": "rows",
         "input_source": "root"}),
    (2, {"transport": "peer", "pipeline": 1, "poison": True, "input_source": "root"}),
    (1, {"pipeline": 1, "poison": True}),
    (1, {"pipeline": 1, "poison": True, "input_source": "root", "lanes": 1}),
])
def test_native_v5_shared_gpu(v5_reference, world, kw):
    """Pipelined chunked V5 through the C ABI (the bench's path) with NaN-poisoned buffers: equal to
    the single-GPU engine to fp32 rounding (Winograd tile origins move with the row split)."""
    y, desc, phases = _run_v5(world, kw)
    y = torch.from_numpy(y)
    err = (y - v5_reference).abs().max().item() / v5_reference.abs().max().item()
    assert err < 1e-5, (err, desc)
    # the layout says whether V5's per-layer halo exchange runs (a batch split has none)
    assert ("none" in desc["halo_exchange"]) == (desc["halo_transfers_per_step"] == 0)
    if world > 1 and kw.get("decomp") == "rows" and kw.get("layer") != "overlap":
        assert desc["halo_transfers_per_step"] > 0 and desc["halo_bytes_per_step"] > 0
    assert desc["transport"] == kw.get("transport", "rccl" if world == 1 else "peer")
    assert desc["input_source"] == kw.get("input_source", "local")
    assert set(phases) == {"scatter", "stage1", "halo_p1", "stage2", "gather", "compute"}
    if kw.get("transport") == "peer":
        assert desc["ordering"] == kw.get("peer_sync", "flags")
    b = desc["bytes_per_step"]
    if desc["input_source"] == "local":  # device-resident: nothing scattered inside a step
        assert sum(b["scatter_recv"]) == 0 and desc["input_placement_bytes"] >= 0
    if world > 1:
        assert b["gather_recv"][0] == sum(b["gather_sent"]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("world,kw", [
    (2, {"decomp": "rows"}),
    (4, {"decomp": "rows", "chunks": 2}),
    (4, {"decomp": "hybrid", "input_source": "root"}),
    (3, {"decomp": "rows", "layer": "overlap", "input_source": "root"}),
    (4, {"decomp": "batch", "input_source": "root", "pipeline": 0}),
])
def test_rccl_transport_loopback_bitwise(v5_reference_direct, world, kw):
    """The RCCL transport's remote path (pack into staging, grouped send / recv, unpack, the second
    communicator for halos chained to the first, after / before events) on ranks sharing the GPU via
    the loopback device comm, pipelined, with every consumed buffer NaN-poisoned: bit-identical to the
    single-GPU engine (direct convolutions), and every rank's transfer log is exactly its record-only
    schedule, step after step."""
    from anx.parallel.workloads import native_schedule
    steps, batch = 4, 6
    kw = {"transport": "loopback", "poison": True, "keep_log": True, **kw}
    res = _run_v5(world, kw, batch=batch, steps=steps, env=DIRECT_ENV, all_ranks=True)
    y, desc, phases, log0 = res[0]
    assert torch.equal(torch.from_numpy(y), v5_reference_direct), desc
    assert desc["transport"] == "rccl-loopback" and "chained" in desc["ordering"]
    src = kw.get("input_source", "local")
    rw = {"rows": world, "hybrid": 0, "batch": 1}[kw["decomp"]]
    layer = kw.get("layer", PER_LAYER)
    for r in range(world):
        log = log0 if r == 0 else res[r]
        one = native_schedule(world, batch, rw, layer, kw.get("chunks", 0), r, "loopback", input_source=src)
        scatter = [l for l in native_schedule(world, batch, rw, layer, kw.get("chunks", 0), r, "loopback",
                                              input_source="root") if l.startswith("scatter")]
        expect = Counter()
        for _ in range(steps):
            expect.update(one)
        if src == "local":  # set_input places the input into both step parities, once
            expect.update(scatter * 2)
        elif kw.get("pipeline", 1):  # the pipeline issues one scatter ahead (step k scatters k+1)
            expect.update(scatter)
        assert Counter(log) == expect, (r, Counter(log) - expect, expect - Counter(log))


@pytest.mark.gpu
def test_v5_local_whole_images_run_lanes(cuda):
    """One rank, 64 images: the whole-image tile runs as 2 free-running lanes of the fused forward (each
    its own engine, stream and tile / output offsets). Both lanes' slices (images 0-31 and 32-63) are
    compared with a one-lane forward of all 64 images."""
    ref = _reference(batch=64)
    y, desc, phases = _run_v5(1, {"pipeline": 1}, batch=64, steps=3)
    assert desc["lane_path"] is True and desc["lanes"] == 2
    y = torch.from_numpy(y)
    assert y.shape == ref.shape
    for lo, hi in ((0, 32), (32, 64)):
        assert y[lo:hi].sub(ref[lo:hi]).abs().max().item() / ref[lo:hi].abs().max().item() < 1e-5, (lo, hi)


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


@pytest.mark.gpu
@pytest.mark.parametrize("root_images", [-1, 48])
def test_native_dp_program_two_ranks_lanes_loopback(cuda, root_images):
    """The dp headline's program natively: two ranks sharing the GPU, each with its own
    whole images placed on its device once (batch split, local input), run as 2 free-running lanes, gathered
    to rank 0 over the RCCL transport's code on the loopback communicator; with root shedding (48: rank 0
    computes 48 images as 2 lanes of 24, rank 1 80 as 2 of 40) or an even split (64 + 64). Bit for bit one
    process's forward of all 128 images: every kernel computes an output element the same way whatever
    batch it is launched with."""
    ref = _reference(batch=128)
    y, desc, phases = _run_v5(2, {"decomp": "batch", "transport": "loopback", "input_source": "local", "lanes": 2,
                                  "pipeline": 1, "root_images": root_images}, batch=128, steps=3)
    y = torch.from_numpy(y)
    assert desc["lane_path"] is True and desc["lanes"] == 2 and desc["row_ways"] == 1
    assert desc["images_per_rank"] == ([64, 64] if root_images < 0 else [48, 80])
    assert desc["halo_exchange"].startswith("none") and desc["transport"].startswith("rccl")
    assert y.shape == ref.shape
    assert torch.equal(y, ref), y.sub(ref).abs().max().item()
    assert phases["gather"] >= 0 and phases["compute"] > 0
