"""Decomposition planner: exact receptive-field rows, Python == C++ planner,
and tile-by-tile execution reproducing the full image for every np (the reference's V2.2/V4
outputs were 14/10 and 8/4 rows instead of 13 at np=2/4 — Appendix A D2/D3)."""
import ctypes as C

import pytest
import torch

from anx import _native as nat
from anx.config import blocks
from anx.models.alexnet_blocks import AlexNetBlocks
from anx.parallel.plan import OVERLAP, PER_LAYER, Rows, make_plan
from anx.utils.init import init_input

# pool2 rows -> conv1 input rows (inclusive)
SURVEY = {
    1: [((0, 12), (0, 226))],
    2: [((0, 6), (0, 146)), ((7, 12), (96, 226))],
    4: [((0, 3), (0, 98)), ((4, 6), (48, 146)), ((7, 9), (96, 194)), ((10, 12), (144, 226))],
    8: [((0, 1), (0, 66)), ((2, 3), (16, 98)), ((4, 5), (48, 130)), ((6, 7), (80, 162)), ((8, 9), (112, 194)),
        ((10, 10), (144, 210)), ((11, 11), (160, 226)), ((12, 12), (176, 226))],
}


@pytest.mark.parametrize("np_", [1, 2, 4, 8])
def test_survey_table(np_):
    p = make_plan(227, 227, np_)
    got = [((t.out.lo, t.out.hi - 1), (t.inp.lo, t.inp.hi - 1)) for t in p.tiles]
    assert got == SURVEY[np_]


def _native_plan(np_, mode):
    b1, b2 = blocks()
    tiles = (nat.TileC * np_)()
    oin = (C.c_int * (2 * np_))()
    op1 = (C.c_int * (2 * np_))()
    cap = 256
    ih, ph = (nat.XferC * cap)(), (nat.XferC * cap)()
    nih, nph = C.c_int(), C.c_int()
    nat.call("anx_make_plan", 227, 227, np_, 0 if mode == OVERLAP else 1, C.byref(nat.block_c(b1)),
             C.byref(nat.block_c(b2)), tiles, oin, op1, ih, C.byref(nih), ph, C.byref(nph), cap)
    return tiles, list(oin), list(op1), [(x.src, x.dst, x.lo, x.hi) for x in ih[:nih.value]], \
        [(x.src, x.dst, x.lo, x.hi) for x in ph[:nph.value]]


@pytest.mark.parametrize("mode", [OVERLAP, PER_LAYER])
@pytest.mark.parametrize("np_", [1, 2, 3, 4, 5, 7, 8, 13, 16])
def test_python_plan_equals_native(np_, mode):
    p = make_plan(227, 227, np_, mode)
    tiles, oin, op1, ih, ph = _native_plan(np_, mode)
    for t, c in zip(p.tiles, tiles):
        assert (t.inp.lo, t.inp.hi, t.c1.lo, t.c1.hi, t.p1.lo, t.p1.hi, t.q.lo, t.q.hi, t.c2.lo, t.c2.hi, t.out.lo,
                t.out.hi) == (c.in_lo, c.in_hi, c.c1_lo, c.c1_hi, c.p1_lo, c.p1_hi, c.q_lo, c.q_hi, c.c2_lo, c.c2_hi,
                              c.out_lo, c.out_hi)
    assert [(r.lo, r.hi) for r in p.owned_in] == [tuple(oin[i:i + 2]) for i in range(0, 2 * np_, 2)]
    assert [(x.src, x.dst, x.rows.lo, x.rows.hi) for x in p.in_halos] == ih
    assert [(x.src, x.dst, x.rows.lo, x.rows.hi) for x in p.p1_halos] == ph


@pytest.mark.parametrize("np_", [2, 4, 8, 16])
def test_owned_rows_partition(np_):
    p = make_plan(227, 227, np_, PER_LAYER)
    live = [r for r in p.owned_in if not r.empty]
    assert live[0].lo == 0 and live[-1].hi == 227
    assert all(a.hi == b.lo for a, b in zip(live, live[1:]))
    p1 = [r for r in p.owned_p1 if not r.empty]
    assert p1[0].lo == 0 and p1[-1].hi == 27 and all(a.hi == b.lo for a, b in zip(p1, p1[1:]))


@pytest.mark.parametrize("np_", [2, 3, 4, 8])
def test_cpu_tiles_reproduce_full_image(np_):
    """Overlap tiles on the host engine concatenate to the single-tile output (bitwise: same code)."""
    m = AlexNetBlocks(device="cpu", init="rand", seed=11)
    x = init_input(1, "rand", seed=11)
    full = m(x)
    p = make_plan(227, 227, np_, OVERLAP)
    parts = [m.tile_forward(x[:, t.inp.lo:t.inp.hi].contiguous(), t) for t in p.tiles if not t.out.empty]
    torch.testing.assert_close(torch.cat(parts, dim=1), full, rtol=0, atol=0)


@pytest.mark.parametrize("np_", [2, 4, 8])
def test_cpu_per_layer_halo_exchange(np_):
    """PER_LAYER: each tile computes only its own pool1 rows, receives pool1 halos from the owners
    (in-process here), and still reproduces the full image."""
    m = AlexNetBlocks(device="cpu", init="rand", seed=12)
    x = init_input(1, "rand", seed=12)
    full = m(x)
    p = make_plan(227, 227, np_, PER_LAYER)
    engines = [AlexNetBlocks(device="cpu", weights=m.weights) for _ in range(np_)]
    for r, t in enumerate(p.tiles):
        if not t.out.empty:
            engines[r].stage1(x[:, t.inp.lo:t.inp.hi].contiguous(), t)
    for h in p.p1_halos:
        rows = engines[h.src].window_get(p.tiles[h.src], h.rows.lo, h.rows.hi, 1)
        engines[h.dst].window_put(p.tiles[h.dst], h.rows.lo, rows)
    parts = [engines[r].stage2(1, t) for r, t in enumerate(p.tiles) if not t.out.empty]
    torch.testing.assert_close(torch.cat(parts, dim=1), full, rtol=0, atol=0)
