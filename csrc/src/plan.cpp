// Exact receptive-field planner (see anx/plan.hpp for the contract and reference citations).
#include "anx/plan.hpp"

#include <algorithm>
#include <cstdio>
#include <string>

namespace anx {

std::vector<RowRange> split_rows(int n, int np) {
  std::vector<RowRange> r(np);
  int lo = 0;
  for (int i = 0; i < np; ++i) {
    const int cnt = n / np + (i < n % np ? 1 : 0);
    r[i] = {lo, lo + cnt};
    lo += cnt;
  }
  return r;
}

static RowRange clip(RowRange r, int lo, int hi) { return {std::max(r.lo, lo), std::min(r.hi, hi)}; }

RowRange conv_rows_needed(RowRange out, int F, int S, int P, int in_rows) {
  if (out.empty()) return {0, 0};
  return clip({out.lo * S - P, (out.hi - 1) * S - P + F}, 0, in_rows);
}

RowRange pool_rows_needed(RowRange out, int F, int S, int in_rows) {
  if (out.empty()) return {0, 0};
  return clip({out.lo * S, (out.hi - 1) * S + F}, 0, in_rows);
}

// Transfers so that every rank t holds `need[t]` given a disjoint ownership `own`.
static std::vector<HaloXfer> halo_xfers(const std::vector<RowRange>& own, const std::vector<RowRange>& need) {
  std::vector<HaloXfer> x;
  const int np = static_cast<int>(own.size());
  for (int dst = 0; dst < np; ++dst) {
    if (need[dst].empty()) continue;
    for (int src = 0; src < np; ++src) {
      if (src == dst || own[src].empty()) continue;
      const RowRange r = clip(need[dst], own[src].lo, own[src].hi);
      if (!r.empty()) x.push_back({src, dst, r});
    }
  }
  return x;
}

DecompPlan make_plan(int H, int W, int np, Decomp mode, const BlockSpec& b1, const BlockSpec& b2) {
  DecompPlan p;
  p.np = np;
  p.mode = mode;
  p.dims = blocks_dims(H, W, b1, b2);
  p.b1 = b1;
  p.b2 = b2;
  const BlocksDims& d = p.dims;
  const auto outs = split_rows(d.Hp2, np);
  p.tiles.resize(np);
  p.owned_p1.resize(np);
  for (int t = 0; t < np; ++t) {
    TilePlan& tp = p.tiles[t];
    tp.out = outs[t];
    if (tp.out.empty()) {
      tp = TilePlan{};
      tp.in = tp.c1 = tp.p1 = tp.q = tp.c2 = tp.out = {0, 0};
      p.owned_p1[t] = {0, 0};
      continue;
    }
    tp.c2 = pool_rows_needed(tp.out, b2.pool.F, b2.pool.S, d.H2);
    // conv2 input window, NOT clipped: rows outside [0,Hp1) are the conv's zero padding.
    tp.q = {tp.c2.lo * b2.conv.S - b2.conv.P, (tp.c2.hi - 1) * b2.conv.S - b2.conv.P + b2.conv.F};
    const RowRange need_p1 = clip(tp.q, 0, d.Hp1);
    if (mode == Decomp::Overlap) {
      tp.p1 = need_p1;
    } else {
      // Own the pool1 rows "under" the owned outputs: [S2*lo, S2*hi), last rank to Hp1.
      const int lo = tp.out.lo * b2.pool.S * b2.conv.S;
      const int hi = (tp.out.hi == d.Hp2) ? d.Hp1 : tp.out.hi * b2.pool.S * b2.conv.S;
      tp.p1 = {lo, std::min(hi, d.Hp1)};
    }
    p.owned_p1[t] = mode == Decomp::PerLayer ? tp.p1 : RowRange{0, 0};
    tp.c1 = pool_rows_needed(tp.p1, b1.pool.F, b1.pool.S, d.H1);
    tp.in = conv_rows_needed(tp.c1, b1.conv.F, b1.conv.S, b1.conv.P, H);
  }
  // Scatter + halo formulation of the input distribution: rank t owns [in_t.lo, in_{t+1}.lo).
  p.owned_in.assign(np, {H, H});
  {
    std::vector<int> live;
    for (int t = 0; t < np; ++t)
      if (!p.tiles[t].out.empty()) live.push_back(t);
    for (size_t i = 0; i < live.size(); ++i) {
      const int t = live[i];
      const int lo = i == 0 ? 0 : p.tiles[t].in.lo;
      const int hi = i + 1 == live.size() ? H : p.tiles[live[i + 1]].in.lo;
      p.owned_in[t] = {lo, std::max(lo, hi)};
    }
  }
  std::vector<RowRange> need_in(np);
  for (int t = 0; t < np; ++t) need_in[t] = p.tiles[t].in;
  p.in_halos = halo_xfers(p.owned_in, need_in);
  if (mode == Decomp::PerLayer) {
    std::vector<RowRange> need_p1(np);
    for (int t = 0; t < np; ++t) need_p1[t] = p.tiles[t].out.empty() ? RowRange{0, 0} : clip(p.tiles[t].q, 0, d.Hp1);
    p.p1_halos = halo_xfers(p.owned_p1, need_p1);
  }
  return p;
}

const char* check_plan(const DecompPlan& p) {
  static thread_local std::string msg;
  const BlocksDims& d = p.dims;
  const ConvSpec& k1 = p.b1.conv;
  const ConvSpec& k2 = p.b2.conv;
  const PoolSpec& q1 = p.b1.pool;
  const PoolSpec& q2 = p.b2.pool;
  int next = 0;
  for (int t = 0; t < p.np; ++t) {
    const TilePlan& tp = p.tiles[t];
    char buf[256];
    if (tp.out.empty()) continue;
    if (tp.out.lo != next) {
      std::snprintf(buf, sizeof buf, "rank %d output rows start at %d, expected %d", t, tp.out.lo, next);
      return (msg = buf).c_str();
    }
    next = tp.out.hi;
    // Layer algebra: each window must produce exactly the next range.
    const int c1_rows = conv_out_dim(tp.in.size(), k1.F, k1.S, 0);
    if (tp.in.lo != tp.c1.lo * k1.S || c1_rows != tp.c1.size()) {
      std::snprintf(buf, sizeof buf, "rank %d conv1 window mismatch", t);
      return (msg = buf).c_str();
    }
    if (tp.c1.lo != tp.p1.lo * q1.S || pool_out_dim(tp.c1.size(), q1.F, q1.S) != tp.p1.size()) {
      std::snprintf(buf, sizeof buf, "rank %d pool1 window mismatch", t);
      return (msg = buf).c_str();
    }
    // stage1 writes the pool1 rows it computes into the conv2 input window at p1.lo - q.lo
    if (tp.p1.lo < tp.q.lo || tp.p1.hi > tp.q.hi) {
      std::snprintf(buf, sizeof buf, "rank %d pool1 rows [%d,%d) outside its conv2 window [%d,%d)", t, tp.p1.lo,
                    tp.p1.hi, tp.q.lo, tp.q.hi);
      return (msg = buf).c_str();
    }
    if (conv_out_dim(tp.q.size(), k2.F, k2.S, 0) != tp.c2.size()) {
      std::snprintf(buf, sizeof buf, "rank %d conv2 window mismatch", t);
      return (msg = buf).c_str();
    }
    if (tp.c2.lo != tp.out.lo * q2.S || pool_out_dim(tp.c2.size(), q2.F, q2.S) != tp.out.size()) {
      std::snprintf(buf, sizeof buf, "rank %d pool2 window mismatch", t);
      return (msg = buf).c_str();
    }
  }
  if (next != d.Hp2) {
    return (msg = "output rows do not cover the image").c_str();
  }
  return "";
}

double conv1_redundancy(const DecompPlan& p) {
  long rows = 0;
  for (const TilePlan& t : p.tiles) rows += t.c1.size();
  return p.dims.H1 > 0 ? static_cast<double>(rows) / p.dims.H1 - 1.0 : 0.0;
}

bool make_hybrid_plan(int H, int W, int np, int batch, int row_ways, Decomp mode, HybridPlan& out,
                      const BlockSpec& b1, const BlockSpec& b2) {
  if (np < 1 || batch < 1 || row_ways < 0 || row_ways > np || (row_ways > 0 && np % row_ways)) return false;
  HybridPlan p;
  p.np = np;
  p.batch = batch;
  if (row_ways > 0) {
    p.groups = np / row_ways;
    p.group_size.assign(p.groups, row_ways);
    p.images = split_rows(batch, p.groups);
  } else if (batch >= np) {
    p.groups = np;
    p.group_size.assign(np, 1);
    p.images = split_rows(batch, np);
  } else {
    p.groups = batch;
    p.images = split_rows(batch, batch);  // one image per group
    for (const RowRange& r : split_rows(np, batch)) p.group_size.push_back(r.size());
  }
  int first = 0;
  for (int g = 0; g < p.groups; ++g) {
    p.group_first.push_back(first);
    for (int j = 0; j < p.group_size[g]; ++j) {
      p.group_of.push_back(g);
      p.index_in_group.push_back(j);
    }
    first += p.group_size[g];
    p.row_plans.push_back(make_plan(H, W, p.group_size[g], mode, b1, b2));
  }
  out = std::move(p);
  return true;
}

double conv1_redundancy(const HybridPlan& p) {
  double rows = 0;
  for (int g = 0; g < p.groups; ++g) rows += (conv1_redundancy(p.row_plans[g]) + 1.0) * p.images[g].size();
  return rows / p.batch - 1.0;
}

}  // namespace anx
