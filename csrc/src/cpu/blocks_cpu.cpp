// Host Blocks 1-2 (see anx/cpu_engine.hpp).
#include <algorithm>
#include <cstring>

#include "anx/cpu_engine.hpp"

namespace anx {

CpuBlocks::CpuBlocks(const BlockSpec& b1, const BlockSpec& b2, int H, int W, const HostWeights& w)
    : b1_(b1), b2_(b2), d_(blocks_dims(H, W, b1, b2)), w_(w), wq_(d_.Wp1 + 2 * b2.conv.P) {}

float* CpuBlocks::window_row(const TilePlan& t, int n, int r) {
  return q_.data() + (static_cast<size_t>(n) * t.q.size() + (r - t.q.lo)) * window_row_floats();
}

void CpuBlocks::stage1(const float* x, int N, const TilePlan& t) {
  const ConvSpec& k1 = b1_.conv;
  q_.assign(static_cast<size_t>(N) * t.q.size() * window_row_floats(), 0.f);
  if (t.out.empty()) return;
  c1_.resize(static_cast<size_t>(N) * t.c1.size() * d_.W1 * d_.C1);
  p1_.resize(static_cast<size_t>(N) * t.p1.size() * d_.Wp1 * d_.C1);
  cpu::conv2d(x, w_.w1.data(), w_.b1.data(), c1_.data(), N, t.in.size(), d_.W, d_.C0, k1.K, k1.F, k1.S, 0, k1.groups,
              true);
  cpu::maxpool(c1_.data(), p1_.data(), N, t.c1.size(), d_.W1, d_.C1, b1_.pool.F, b1_.pool.S);
  // place pool1 rows into the zero-bordered window
  const int P = b2_.conv.P;
  for (int n = 0; n < N; ++n)
    for (int r = t.p1.lo; r < t.p1.hi; ++r)
      std::memcpy(window_row(t, n, r) + static_cast<size_t>(P) * d_.C1,
                  p1_.data() + (static_cast<size_t>(n) * t.p1.size() + (r - t.p1.lo)) * d_.Wp1 * d_.C1,
                  sizeof(float) * d_.Wp1 * d_.C1);
}

void CpuBlocks::stage2(int N, const TilePlan& t, float* y) {
  if (t.out.empty()) return;
  const ConvSpec& k2 = b2_.conv;
  c2_.resize(static_cast<size_t>(N) * t.c2.size() * d_.W2 * d_.C2);
  // window already carries H and W padding
  cpu::conv2d(q_.data(), w_.w2.data(), w_.b2.data(), c2_.data(), N, t.q.size(), wq_, d_.C1, k2.K, k2.F, k2.S, 0,
              k2.groups, true);
  if (b2_.has_lrn) {
    p2_.resize(static_cast<size_t>(N) * t.out.size() * d_.Wp2 * d_.C2);
    cpu::maxpool(c2_.data(), p2_.data(), N, t.c2.size(), d_.W2, d_.C2, b2_.pool.F, b2_.pool.S);
    const LrnSpec& l = b2_.lrn;
    cpu::lrn(p2_.data(), y, N, t.out.size(), d_.Wp2, d_.C2, l.N, l.alpha, l.beta, l.k, l.mode);
  } else {
    cpu::maxpool(c2_.data(), y, N, t.c2.size(), d_.W2, d_.C2, b2_.pool.F, b2_.pool.S);
  }
}

void CpuBlocks::tile_forward(const float* x, int N, const TilePlan& t, float* y) {
  stage1(x, N, t);
  stage2(N, t, y);
}

void CpuBlocks::forward(const float* x, int N, float* y) {
  const DecompPlan p = make_plan(d_.H, d_.W, 1, Decomp::Overlap, b1_, b2_);
  tile_forward(x, N, p.tiles[0], y);
}

}  // namespace anx
