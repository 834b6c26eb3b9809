// CPU reference layers (V1 serial path and the host-side golden oracle).
//
// Same math as the reference's serialConvLayer / serialReluLayer / serialMaxPoolLayer /
// serialLRNLayer (v1_serial/src/layers_serial.cpp:37-175) extended with a batch axis,
// groups and per-edge row padding. The conv is reorganised for the host cache: weights are
// transposed once to [g][fh][fw][c][k] so the innermost loop is a contiguous, vectorisable
// axpy over output channels — numerically a different summation order than the reference's
// c->fh->fw loop, so oracle comparisons use a relative tolerance, not bit equality.
#include <algorithm>
#include <cmath>
#include <limits>
#include <vector>

#include "anx/ops.hpp"

namespace anx::cpu {

void conv2d(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C, int K, int F,
            int S, int P, int groups, bool relu, int pad_top, int pad_bottom) {
  const int pt = pad_top < 0 ? P : pad_top;
  const int pb = pad_bottom < 0 ? P : pad_bottom;
  const int Ho = conv_out_dim(H + pt + pb, F, S, 0);
  const int Wo = conv_out_dim(W, F, S, P);
  const int Cg = C / groups, Kg = K / groups;
  // [g][fh][fw][c][kk]
  std::vector<float> wt(static_cast<size_t>(groups) * F * F * Cg * Kg);
  for (int g = 0; g < groups; ++g)
    for (int kk = 0; kk < Kg; ++kk)
      for (int c = 0; c < Cg; ++c)
        for (int fh = 0; fh < F; ++fh)
          for (int fw = 0; fw < F; ++fw) {
            const int k = g * Kg + kk;
            wt[((((static_cast<size_t>(g) * F + fh) * F + fw) * Cg + c) * Kg) + kk] =
                w[((static_cast<size_t>(k) * Cg + c) * F + fh) * F + fw];
          }
  std::vector<float> acc(Kg);
  for (int n = 0; n < N; ++n)
    for (int oy = 0; oy < Ho; ++oy)
      for (int ox = 0; ox < Wo; ++ox)
        for (int g = 0; g < groups; ++g) {
          for (int kk = 0; kk < Kg; ++kk) acc[kk] = b ? b[g * Kg + kk] : 0.f;
          for (int fh = 0; fh < F; ++fh) {
            const int iy = oy * S + fh - pt;
            if (iy < 0 || iy >= H) continue;
            for (int fw = 0; fw < F; ++fw) {
              const int ix = ox * S + fw - P;
              if (ix < 0 || ix >= W) continue;
              const float* xp = x + nhwc(n, iy, ix, g * Cg, H, W, C);
              const float* wp = wt.data() + ((static_cast<size_t>(g) * F + fh) * F + fw) * Cg * Kg;
              for (int c = 0; c < Cg; ++c) {
                const float xv = xp[c];
                const float* wr = wp + static_cast<size_t>(c) * Kg;
                for (int kk = 0; kk < Kg; ++kk) acc[kk] += xv * wr[kk];
              }
            }
          }
          float* yp = y + nhwc(n, oy, ox, g * Kg, Ho, Wo, K);
          for (int kk = 0; kk < Kg; ++kk) yp[kk] = relu ? std::max(acc[kk], 0.f) : acc[kk];
        }
}

void relu(float* x, size_t n) {
  for (size_t i = 0; i < n; ++i) x[i] = std::max(x[i], 0.f);
}

void maxpool(const float* x, float* y, int N, int H, int W, int C, int F, int S) {
  const int Ho = pool_out_dim(H, F, S), Wo = pool_out_dim(W, F, S);
  for (int n = 0; n < N; ++n)
    for (int oy = 0; oy < Ho; ++oy)
      for (int ox = 0; ox < Wo; ++ox) {
        float* yp = y + nhwc(n, oy, ox, 0, Ho, Wo, C);
        for (int c = 0; c < C; ++c) yp[c] = -std::numeric_limits<float>::infinity();
        for (int fh = 0; fh < F; ++fh)
          for (int fw = 0; fw < F; ++fw) {
            const int iy = oy * S + fh, ix = ox * S + fw;
            if (iy >= H || ix >= W) continue;
            const float* xp = x + nhwc(n, iy, ix, 0, H, W, C);
            for (int c = 0; c < C; ++c) yp[c] = std::max(yp[c], xp[c]);
          }
      }
}

void lrn(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta, float k,
         LrnMode mode) {
  const float a = mode == LrnMode::DivN ? alpha / static_cast<float>(size) : alpha;
  const int half = size / 2;
  const size_t P = static_cast<size_t>(N) * H * W;
  for (size_t p = 0; p < P; ++p) {
    const float* xp = x + p * C;
    float* yp = y + p * C;
    for (int c = 0; c < C; ++c) {
      float s = 0.f;
      const int lo = std::max(0, c - half), hi = std::min(C - 1, c + half);
      for (int j = lo; j <= hi; ++j) s += xp[j] * xp[j];
      yp[c] = xp[c] / std::pow(k + a * s, beta);
    }
  }
}

}  // namespace anx::cpu
