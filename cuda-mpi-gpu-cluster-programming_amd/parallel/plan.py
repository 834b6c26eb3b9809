"""Exact receptive-field decomposition planner (Python mirror of csrc/src/plan.cpp).

The reference sizes halos as F/2 rows and trims with ad-hoc formulas
(final_project/v2_mpi_only/2.2_scatter_halo/src/main.cpp:119-230,
final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:65-122), so its np>=2 outputs have 14/10 or 8/4
rows instead of 13. This planner partitions the 13 OUTPUT rows
and back-propagates the receptive field pool2 -> conv2 -> pool1 -> conv1, as the reference's unused
``mapRangeStart/mapRangeEnd`` tried to (v4_mpi_cuda/src/alexnet_mpi_cuda.cu:27-83).

All ranges are half-open [lo, hi) in the global row index of the named layer.
``tests/test_plan.py`` checks this against the C++ planner (``anx_make_plan``) row by row.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ..config import BLOCK1, BLOCK2, BlockSpec, blocks_dims, conv_out_dim, pool_out_dim

OVERLAP, PER_LAYER = "overlap", "per_layer"


@dataclass(frozen=True)
class Rows:
    lo: int = 0
    hi: int = 0

    @property
    def size(self) -> int:
        return max(0, self.hi - self.lo)

    @property
    def empty(self) -> bool:
        return self.hi <= self.lo

    def clip(self, lo: int, hi: int) -> "Rows":
        return Rows(max(self.lo, lo), min(self.hi, hi))


EMPTY = Rows(0, 0)


@dataclass(frozen=True)
class TilePlan:
    inp: Rows  # input image rows read
    c1: Rows   # conv1 rows computed
    p1: Rows   # pool1 rows computed locally
    q: Rows    # conv2 input window (pool1 index space; outside [0,Hp1) = zero padding)
    c2: Rows   # conv2 rows computed
    out: Rows  # pool2/LRN rows produced (owned)


EMPTY_TILE = TilePlan(EMPTY, EMPTY, EMPTY, EMPTY, EMPTY, EMPTY)


@dataclass(frozen=True)
class Xfer:
    src: int
    dst: int
    rows: Rows


@dataclass
class DecompPlan:
    np: int
    mode: str
    H: int
    W: int
    tiles: list = field(default_factory=list)
    owned_in: list = field(default_factory=list)
    in_halos: list = field(default_factory=list)
    owned_p1: list = field(default_factory=list)
    p1_halos: list = field(default_factory=list)


def split_rows(n: int, np_: int) -> list[Rows]:
    """First n % np ranks get one extra row (the reference's Scatterv rule,
    v2_mpi_only/2.2_scatter_halo/src/main.cpp:102-109)."""
    out, lo = [], 0
    for i in range(np_):
        cnt = n // np_ + (1 if i < n % np_ else 0)
        out.append(Rows(lo, lo + cnt))
        lo += cnt
    return out


def conv_rows_needed(out: Rows, F: int, S: int, P: int, in_rows: int) -> Rows:
    if out.empty:
        return EMPTY
    return Rows(out.lo * S - P, (out.hi - 1) * S - P + F).clip(0, in_rows)


def pool_rows_needed(out: Rows, F: int, S: int, in_rows: int) -> Rows:
    if out.empty:
        return EMPTY
    return Rows(out.lo * S, (out.hi - 1) * S + F).clip(0, in_rows)


def _halo_xfers(own: list[Rows], need: list[Rows]) -> list[Xfer]:
    xs = []
    for dst, nd in enumerate(need):
        if nd.empty:
            continue
        for src, ow in enumerate(own):
            if src == dst or ow.empty:
                continue
            r = nd.clip(ow.lo, ow.hi)
            if not r.empty:
                xs.append(Xfer(src, dst, r))
    return xs


def make_plan(H: int, W: int, np_: int, mode: str = OVERLAP, b1: BlockSpec = BLOCK1,
              b2: BlockSpec = BLOCK2) -> DecompPlan:
    if np_ < 1:
        raise ValueError("np must be >= 1")
    if mode not in (OVERLAP, PER_LAYER):
        raise ValueError(f"mode must be {OVERLAP!r} or {PER_LAYER!r}")
    d = blocks_dims(H, W, b1, b2)
    p = DecompPlan(np_, mode, H, W)
    for out in split_rows(d.Hp2, np_):
        if out.empty:
            p.tiles.append(EMPTY_TILE)
            p.owned_p1.append(EMPTY)
            continue
        c2 = pool_rows_needed(out, b2.pool.F, b2.pool.S, d.H2)
        q = Rows(c2.lo * b2.conv.S - b2.conv.P, (c2.hi - 1) * b2.conv.S - b2.conv.P + b2.conv.F)
        if mode == OVERLAP:
            p1 = q.clip(0, d.Hp1)
        else:
            step = b2.pool.S * b2.conv.S
            hi = d.Hp1 if out.hi == d.Hp2 else out.hi * step
            p1 = Rows(out.lo * step, min(hi, d.Hp1))
        p.owned_p1.append(p1 if mode == PER_LAYER else EMPTY)
        c1 = pool_rows_needed(p1, b1.pool.F, b1.pool.S, d.H1)
        inp = conv_rows_needed(c1, b1.conv.F, b1.conv.S, b1.conv.P, H)
        p.tiles.append(TilePlan(inp, c1, p1, q, c2, out))
    live = [t for t in range(np_) if not p.tiles[t].out.empty]
    p.owned_in = [Rows(H, H)] * np_
    for i, t in enumerate(live):
        lo = 0 if i == 0 else p.tiles[t].inp.lo
        hi = H if i + 1 == len(live) else p.tiles[live[i + 1]].inp.lo
        p.owned_in[t] = Rows(lo, max(lo, hi))
    p.in_halos = _halo_xfers(p.owned_in, [t.inp for t in p.tiles])
    if mode == PER_LAYER:
        need = [EMPTY if t.out.empty else t.q.clip(0, d.Hp1) for t in p.tiles]
        p.p1_halos = _halo_xfers(p.owned_p1, need)
    check_plan(p, b1, b2)
    return p


def conv1_redundancy(p: DecompPlan, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> float:
    """Conv1 rows computed by all ranks / the image's conv1 rows - 1 (0 = nothing recomputed)."""
    d = blocks_dims(p.H, p.W, b1, b2)
    return sum(t.c1.size for t in p.tiles) / d.H1 - 1.0


@dataclass
class HybridPlan:
    """Batch x rows decomposition (mirror of anx::make_hybrid_plan, csrc/src/plan.cpp): ``groups``
    groups of contiguous ranks; group g computes images ``images[g]`` row-decomposed over its
    ``group_size[g]`` ranks by ``row_plans[g]``."""
    np: int
    batch: int
    groups: int
    images: list
    group_size: list
    group_of: list
    index_in_group: list
    row_plans: list

    def tile(self, rank: int) -> TilePlan:
        return self.row_plans[self.group_of[rank]].tiles[self.index_in_group[rank]]

    def images_of(self, rank: int) -> Rows:
        return self.images[self.group_of[rank]]

    def group_ranks(self, g: int) -> list[int]:
        first = sum(self.group_size[:g])
        return list(range(first, first + self.group_size[g]))


def make_hybrid_plan(H: int, W: int, np_: int, batch: int, row_ways: int = 0, mode: str = OVERLAP,
                     b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> HybridPlan:
    """Split the batch across ranks first, rows only where there are fewer images than ranks
    (``row_ways=0``), or ``row_ways`` ranks per image group when asked (``row_ways=np``: the
    reference's pure row split, v2_mpi_only/2.2_scatter_halo/src/main.cpp:100-249)."""
    if np_ < 1 or batch < 1 or row_ways < 0 or row_ways > np_ or (row_ways and np_ % row_ways):
        raise ValueError(f"invalid hybrid plan: np={np_} batch={batch} row_ways={row_ways}")
    if row_ways:
        groups = np_ // row_ways
        sizes = [row_ways] * groups
        images = split_rows(batch, groups)
    elif batch >= np_:
        groups, sizes, images = np_, [1] * np_, split_rows(batch, np_)
    else:
        groups = batch
        images = split_rows(batch, batch)
        sizes = [r.size for r in split_rows(np_, batch)]
    group_of, index = [], []
    for g, n in enumerate(sizes):
        group_of += [g] * n
        index += list(range(n))
    plans = [make_plan(H, W, n, mode, b1, b2) for n in sizes]
    return HybridPlan(np_, batch, groups, images, sizes, group_of, index, plans)


def hybrid_conv1_redundancy(p: HybridPlan, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> float:
    rows = sum((conv1_redundancy(rp, b1, b2) + 1.0) * im.size for rp, im in zip(p.row_plans, p.images))
    return rows / p.batch - 1.0


def full_plan(H: int, W: int, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> TilePlan:
    return make_plan(H, W, 1, OVERLAP, b1, b2).tiles[0]


def check_plan(p: DecompPlan, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2) -> None:
    """Raise ValueError unless the tiles partition the output rows and every layer window matches the
    layer algebra (the C++ check_plan's contract; no ``assert``, so ``python -O`` keeps the checks)."""
    d = blocks_dims(p.H, p.W, b1, b2)
    nxt = 0

    def need(ok: bool, msg: str) -> None:
        if not ok:
            raise ValueError(msg)

    for r, t in enumerate(p.tiles):
        if t.out.empty:
            continue
        need(t.out.lo == nxt, f"rank {r}: output rows start at {t.out.lo}, expected {nxt}")
        nxt = t.out.hi
        need(t.inp.lo == t.c1.lo * b1.conv.S and conv_out_dim(t.inp.size, b1.conv.F, b1.conv.S, 0) == t.c1.size,
             f"rank {r}: conv1 window")
        need(t.c1.lo == t.p1.lo * b1.pool.S and pool_out_dim(t.c1.size, b1.pool.F, b1.pool.S) == t.p1.size,
             f"rank {r}: pool1 window")
        # the pool1 rows a rank computes land inside its conv2 input window (stage1 writes them there)
        need(t.q.lo <= t.p1.lo and t.p1.hi <= t.q.hi, f"rank {r}: pool1 rows outside the conv2 window")
        need(conv_out_dim(t.q.size, b2.conv.F, b2.conv.S, 0) == t.c2.size, f"rank {r}: conv2 window")
        need(t.c2.lo == t.out.lo * b2.pool.S and pool_out_dim(t.c2.size, b2.pool.F, b2.pool.S) == t.out.size,
             f"rank {r}: pool2 window")
    need(nxt == d.Hp2, "output rows do not cover the image")


# ----------------------------------------------------------------------------- V5 step schedule
# Mirror of anx::plan_stats / make_v5_layout (csrc/src/runtime/v5.cpp) and of
# anx::make_step_schedule / chunk_of (csrc/src/runtime/schedule.cpp): tests/test_v5_runtime.py checks
# that the native runtime issues exactly this transfer list.

MAX_CHUNKS = 16


def plan_stats(p: HybridPlan) -> dict:
    """Per-rank work balance: output rows (max / mean) and images x rows (imbalance = max / mean)."""
    rows = [p.tile(r).out.size for r in range(p.np)]
    imgs = [p.images_of(r).size if rows[r] else 0 for r in range(p.np)]
    work = [a * b for a, b in zip(rows, imgs)]
    mean = sum(work) / p.np
    return {"groups": p.groups, "row_ways": max(p.group_size), "out_rows_max": max(rows),
            "out_rows_mean": sum(rows) / p.np, "imbalance": max(work) / mean if mean else 1.0,
            "conv1_redundancy": hybrid_conv1_redundancy(p), "images_per_rank_max": max(imgs)}


def pick_row_ways(np_: int, batch: int, workload: str = "v5", input_source: str = "local",
                  mode: str = PER_LAYER) -> int:
    """The runtimes' default row split: the native cost model's lowest modelled step over the divisors
    of np (anx/cost.hpp; :mod:`anx.parallel.cost`)."""
    from .cost import pick_row_ways as native_pick
    return native_pick(workload, np_, batch, input_source, "per_layer" if mode == PER_LAYER else "overlap")


def _xfer(phase, src, dst, frm, to, width, height):
    return (f"{phase} {src}->{dst} w={width} h={height} from={frm[0]}+{frm[1]}/{frm[2]} "
            f"to={to[0]}+{to[1]}/{to[2]}")


def step_schedule(p: HybridPlan, chunks: int = 0, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2,
                  input_source: str = "root") -> list[str]:
    """Every transfer of one V5 step in issue order (scatter with root input, pool1-halo chunks,
    gather), in the native Transfer::str() format: a 2-D block of `h` images x `w` bytes between buffer
    regions (X / Tile / Win / Y / YFull + byte offset / image pitch). With local input the scatter is
    the one-time placement of set_input, not part of a step."""
    d = blocks_dims(p.row_plans[0].H, p.row_plans[0].W, b1, b2)
    in_row, out_row = d.W * d.C0 * 4, d.Wp2 * d.C2 * 4
    win_row = (d.Wp1 + 2 * b2.conv.P) * d.C1 * 4
    scatter, gather, halos = [], [], []
    for q in range(p.np):
        t, im = p.tile(q), p.images_of(q)
        if t.out.empty or im.empty:
            continue
        scatter.append(("scatter", 0, q, ("X", (im.lo * d.H + t.inp.lo) * in_row, d.H * in_row),
                        ("Tile", 0, t.inp.size * in_row), t.inp.size * in_row, im.size))
        gather.append(("gather", q, 0, ("Y", 0, t.out.size * out_row),
                       ("YFull", (im.lo * d.Hp2 + t.out.lo) * out_row, d.Hp2 * out_row), t.out.size * out_row,
                       im.size))
    for g, rp in enumerate(p.row_plans):
        base, n = sum(p.group_size[:g]), p.images[g].size
        if n == 0:
            continue
        for h in rp.p1_halos:
            ts, td = rp.tiles[h.src], rp.tiles[h.dst]
            halos.append(("halo_p1", base + h.src, base + h.dst,
                          ("Win", (h.rows.lo - ts.q.lo) * win_row, ts.q.size * win_row),
                          ("Win", (h.rows.lo - td.q.lo) * win_row, td.q.size * win_row), h.rows.size * win_row, n))
    if halos:
        least = min(x[6] for x in halos)
        chunks = max(1, min(chunks if chunks > 0 else 1, least, MAX_CHUNKS))  # auto: 1 (the runtime's rule)
    out = [_xfer(*x) for x in scatter] if input_source == "root" else []
    for c in range(chunks if halos else 0):
        for ph, s, t, frm, to, w, hgt in halos:
            lo, hi = hgt * c // chunks, hgt * (c + 1) // chunks
            if hi > lo:
                out.append(_xfer(f"{ph}#{c}", s, t, (frm[0], frm[1] + lo * frm[2], frm[2]),
                                 (to[0], to[1] + lo * to[2], to[2]), w, hi - lo))
    return out + [_xfer(*x) for x in gather]
