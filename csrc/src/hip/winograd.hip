// Winograd F(3x3, 5x5) and F(4x4, 5x5) convolution for stride-1 5x5 layers (AlexNet Conv2), fp32 end
// to end (WinoPlan::m = 3 or 4; the 4x4 tiles: 64 points per 16 outputs, wino_gemm16.hpp).
//
//   Y = A^T [ U (.) V ] A,  U = G g G^T (49 x C x K, once per weight set, host fp64 -> fp32),
//                           V = B^T d B (per 7x7 input tile and channel), 3x3 outputs per tile.
// 49 multiplies per 9 outputs instead of 225: Conv2's 896 MFLOP/image become 195 MFLOP/image of
// MFMA work. The reference has no fast-convolution algorithm (direct loops everywhere:
// v3_cuda_only/src/layers_cuda.cu:20-46). fp32 error of this point set is ~5e-7 of sum|terms|
// (tools/winograd_numerics.py), the same order as the fp32 accumulation error of the direct sum.
//
// Two launches, both on the caller's stream:
//   1. input transform : window [N][Hq][Wq][C] -> V [P][49][C]   (VALU, 2 channels per thread)
//   2. fused batched GEMM + output transform + bias + ReLU (wino_gemm.hpp): M = V . U never leaves
//      registers, Y goes straight to the NHWC conv output.
#include <hip/hip_runtime.h>

#include <vector>

#include "anx/ops.hpp"
#include "anx/winograd_f35.hpp"
#include "anx/winograd_f45.hpp"

namespace anx::hip {
namespace {

using f32x2 = __attribute__((ext_vector_type(2))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kT = 256;

// The two tile sizes (WinoPlan::m): F(3x3,5x5) -> 3x3 outputs from 7x7 inputs, F(4x4,5x5) -> 4x4 from 8x8.
template <int M>
struct WT;
template <>
struct WT<3> {
  static constexpr int kM = 3, kN = 7;
  static constexpr float bt(int a, int u) { return wino::kBT[a][u]; }
  static constexpr double g(int a, int u) { return wino::kG[a][u]; }
};
template <>
struct WT<4> {
  static constexpr int kM = 4, kN = 8;
  static constexpr float bt(int a, int u) { return wino45::kBT[a][u]; }
  static constexpr double g(int a, int u) { return wino45::kG[a][u]; }
};
constexpr int npt(int m) { return (m + 4) * (m + 4); }

// Thread = (tile, 2 channels): consecutive threads read consecutive channel pairs (coalesced NHWC
// 8-B loads and stores); the 7x7 patch streams through t = B^T d one input row at a time. 98
// transform registers keep 3+ waves per SIMD. C even.
template <int M>
__global__ void __launch_bounds__(kT) wino_in2_kernel(const float* __restrict__ x, float* __restrict__ V, int N, int Hq,
                                                      int Wq, int C, int ty, int tx) {
  using T = WT<M>;
  constexpr int kN = T::kN, kM = T::kM;
  const int C2 = C >> 1;
  // 32-bit index math (total < 2^31, checked by the launcher): 64-bit divisions cost more than the loads
  const int total = N * ty * tx * C2;
  for (int i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    const int c = (i % C2) * 2;
    const int p = i / C2;
    const int tj = p % tx;
    const int q = p / tx;
    const int ti = q % ty;
    const int n = q / ty;
    f32x2 t[kN][kN];
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int v = 0; v < kN; ++v) t[a][v] = f32x2{0.f, 0.f};
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int yy = ti * kM + u;
      f32x2 row[kN];
#pragma unroll
      for (int v = 0; v < kN; ++v) {
        const int xx = tj * kM + v;
        row[v] = (yy < Hq && xx < Wq)
                     ? *reinterpret_cast<const f32x2*>(x + ((static_cast<size_t>(n) * Hq + yy) * Wq + xx) * C + c)
                     : f32x2{0.f, 0.f};
      }
#pragma unroll
      for (int a = 0; a < kN; ++a)
        if (T::bt(a, u) != 0.f)
#pragma unroll
          for (int v = 0; v < kN; ++v) {  // per-component fmaf (no packed FMA): the transform's rounding
            t[a][v].x = fmaf(T::bt(a, u), row[v].x, t[a][v].x);
            t[a][v].y = fmaf(T::bt(a, u), row[v].y, t[a][v].y);
          }
    }
    float* out = V + static_cast<size_t>(p) * (kN * kN) * C + c;
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int b = 0; b < kN; ++b) {
        f32x2 s2 = {0.f, 0.f};
#pragma unroll
        for (int v = 0; v < kN; ++v)
          if (T::bt(b, v) != 0.f) {
            s2.x = fmaf(T::bt(b, v), t[a][v].x, s2.x);
            s2.y = fmaf(T::bt(b, v), t[a][v].y, s2.y);
          }
        *reinterpret_cast<f32x2*>(out + static_cast<size_t>(a * kN + b) * C) = s2;
      }
  }
}

// Pool1 (3x3 / 2 max) fused with the input transform: the conv2 window is never written. One
// workgroup = (image, tile row, 32-channel group): it pools the 7 window rows of its tile row
// straight from the conv1 output into LDS (zero border included), runs t = B^T d down each of the
// window's columns in place, then B along each tile's 7 columns, and writes V. The fmaf sequences are
// those of wino_in2_kernel (same zero skips, same order) and max is exact in any order, so V is
// bit-identical to pool1 + wino_in2. The workgroups of one (image, channel group) share conv1 rows between adjacent
// tile rows: they get equal blockIdx % 8 (one XCD under round-robin dispatch), so re-reads hit that
// XCD's L2.
constexpr int kMaxWq = 31;  // window columns held in LDS
// POOL = false: the same kernel on a materialised conv2 window (`c1` = window [N][Hq][Wq][C], q_lo, Hp,
// Wp, P, c1_lo unused): the window rows of the tile row are copied to LDS with 16-B loads (each
// window row read once per tile row instead of once per tile it touches, as wino_in2_kernel does).
// MERGE (with POOL = false): the window's pool1 pixels came from conv1_fused_pool, which leaves the
// partial max of a window straddling two Conv1 workgroups in p1 ([N][Hp][Wp][C], images from n_off in
// the Conv1 launch's tile numbering of ty1 x tx1 tiles per image; q_lo / P / Hp / Wp locate the pool1
// image in the window): those pixels are max(window, p1), the rest the window's value.
template <int M, int kPG, int NT, bool POOL = true, bool MERGE = false>  // tile, channels, threads per workgroup
__global__ void __launch_bounds__(NT) pool_wino_in_kernel(const float* __restrict__ c1, float* __restrict__ V, int groups,
                                                          int H1, int W1, int C, int Hq, int Wq, int q_lo, int Hp,
                                                          int Wp, int P, int c1_lo, int ty, int tx,
                                                          const float* __restrict__ p1 = nullptr, int n_off = 0,
                                                          int ty1 = 0, int tx1 = 0) {
  using T = WT<M>;
  constexpr int kN = T::kN, kM = T::kM;
  __shared__ __attribute__((aligned(16))) float band[kN][kMaxWq][kPG];
  const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
  const int grp = (j / ty) * 8 + xcd, ti = j % ty;
  if (grp >= groups) return;  // whole workgroup, before any barrier
  const int CG = C / kPG, n = grp / CG, cg = grp % CG;
  const int tid = threadIdx.x;
  // 1. pooled window rows 3ti .. 3ti+6 into LDS, zero outside the pooled image. A thread owns one
  // (pooled column, 4-channel group) of the band's upper (rows 0-3) or lower (rows 4-6) half: the row
  // max of each conv1 row its pooled rows touch (3 loads) is reused by the two pooled rows that share
  // that conv1 row. Two halves: every thread of the 512 has a walk, each walk half as long.
  if constexpr (!POOL) {
    for (int it = tid; it < kN * Wq * (kPG / 4); it += NT) {
      const int c4 = it % (kPG / 4), rest = it / (kPG / 4), col = rest % Wq, r = rest / Wq;
      const int R = ti * kM + r;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (R < Hq)
        v = *reinterpret_cast<const f32x4*>(c1 + (static_cast<size_t>(n * Hq + R) * Wq + col) * C + cg * kPG + 4 * c4);
      if constexpr (MERGE) {
        const int pr = q_lo + R, pc = col - P;
        if (R < Hq && pr >= 0 && pr < Hp && pc >= 0 && pc < Wp && pool1_straddles(n + n_off, pr, pc, ty1, tx1)) {
          const f32x4 u =
              *reinterpret_cast<const f32x4*>(p1 + (static_cast<size_t>(n * Hp + pr) * Wp + pc) * C + cg * kPG + 4 * c4);
          v = f32x4{fmaxf(v.x, u.x), fmaxf(v.y, u.y), fmaxf(v.z, u.z), fmaxf(v.w, u.w)};
        }
      }
      *reinterpret_cast<f32x4*>(&band[r][col][4 * c4]) = v;
    }
  }
  const int per_half = Wq * (kPG / 4);
  for (int it = tid; it < (POOL ? 2 * per_half : 0); it += NT) {
    const int half = it / per_half, ih = it - half * per_half;
    const int r0 = half ? 4 : 0, r1 = half ? kN : 4;
    const int c4 = ih % (kPG / 4), col = ih / (kPG / 4), pc = col - P;
    const bool cin = pc >= 0 && pc < Wp;
    const float* src = c1 + (static_cast<size_t>(n * H1) * W1 + 2 * pc) * C + cg * kPG + 4 * c4;
    f32x4 prev = {0.f, 0.f, 0.f, 0.f};  // row max of conv1 row 2*pr (shared with pooled row pr - 1)
    int prev_row = -1;
#pragma unroll
    for (int r = 0; r < kN; ++r) {
      if (r < r0 || r >= r1) continue;
      const int R = ti * kM + r, pr = q_lo + R;
      f32x4 m = {0.f, 0.f, 0.f, 0.f};
      if (cin && R < Hq && pr >= 0 && pr < Hp) {
        f32x4 h[3];
#pragma unroll
        for (int fh = 0; fh < 3; ++fh) {
          const int cr = 2 * pr + fh - c1_lo;  // local conv1 row
          if (fh == 0 && cr == prev_row) {
            h[0] = prev;
            continue;
          }
          const float* q = src + static_cast<size_t>(cr) * W1 * C;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(q), v1 = *reinterpret_cast<const f32x4*>(q + C),
                      v2 = *reinterpret_cast<const f32x4*>(q + 2 * C);
          h[fh] = f32x4{fmaxf(fmaxf(v0.x, v1.x), v2.x), fmaxf(fmaxf(v0.y, v1.y), v2.y), fmaxf(fmaxf(v0.z, v1.z), v2.z),
                        fmaxf(fmaxf(v0.w, v1.w), v2.w)};
        }
        prev = h[2];
        prev_row = 2 * pr + 2 - c1_lo;
        m = f32x4{fmaxf(fmaxf(h[0].x, h[1].x), h[2].x), fmaxf(fmaxf(h[0].y, h[1].y), h[2].y),
                  fmaxf(fmaxf(h[0].z, h[1].z), h[2].z), fmaxf(fmaxf(h[0].w, h[1].w), h[2].w)};
      }
      *reinterpret_cast<f32x4*>(&band[r][col][4 * c4]) = m;
    }
  }
  __syncthreads();
  // 2. t = B^T d down each column, in place (a thread owns one (column, 4-channel group))
  for (int it = tid; it < Wq * (kPG / 4); it += NT) {
    const int c4 = it % (kPG / 4), col = it / (kPG / 4);
    f32x4 d[kN], t[kN];
#pragma unroll
    for (int u = 0; u < kN; ++u) d[u] = *reinterpret_cast<const f32x4*>(&band[u][col][4 * c4]);
#pragma unroll
    for (int a = 0; a < kN; ++a) {
      t[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < kN; ++u)
        if (T::bt(a, u) != 0.f)
#pragma unroll
          for (int e = 0; e < 4; ++e) t[a][e] = fmaf(T::bt(a, u), d[u][e], t[a][e]);
    }
#pragma unroll
    for (int a = 0; a < kN; ++a) *reinterpret_cast<f32x4*>(&band[a][col][4 * c4]) = t[a];
  }
  __syncthreads();
  // 3. V[a][b] = sum_v B^T[b][v] t[a][3tj + v], one (tile, row a, 4-channel group) per thread: 16-B stores
  for (int it = tid; it < tx * kN * (kPG / 4); it += NT) {
    const int c4 = it % (kPG / 4), rest = it / (kPG / 4), a = rest % kN, tj = rest / kN;
    f32x4 t[kN];
#pragma unroll
    for (int v = 0; v < kN; ++v)
      t[v] = tj * kM + v < Wq ? *reinterpret_cast<const f32x4*>(&band[a][tj * kM + v][4 * c4]) : f32x4{0.f, 0.f, 0.f, 0.f};
    const int p = (n * ty + ti) * tx + tj;
    float* out = V + (static_cast<size_t>(p) * (kN * kN) + a * kN) * C + cg * kPG + 4 * c4;
#pragma unroll
    for (int bb = 0; bb < kN; ++bb) {
      f32x4 s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < kN; ++v)
        if (T::bt(bb, v) != 0.f)
#pragma unroll
          for (int e = 0; e < 4; ++e) s1[e] = fmaf(T::bt(bb, v), t[v][e], s1[e]);
      *reinterpret_cast<f32x4*>(out + static_cast<size_t>(bb) * C) = s1;
    }
  }
}

}  // namespace

hipError_t wino_pool_input(const WinoPlan& w, const float* c1, int H1, int W1, int q_lo, int Hp, int Wp, int P,
                           int c1_lo, float* V, hipStream_t s, int pool_F, int pool_S) {
  constexpr int pg = 32;
  if (pool_F != 3 || pool_S != 2) return hipErrorInvalidValue;  // the walk below is 3x3 / stride 2 only  // 16 channels (14 KiB of LDS) ran slower under lanes: profiles/r03_transform_lds_*
  if (w.C % pg || w.Wq > kMaxWq || static_cast<long>(w.P) * w.C * npt(w.m) >= (1L << 31)) return hipErrorInvalidValue;
  if (w.P == 0) return hipSuccess;
  const int groups = w.N * (w.C / pg);
  const unsigned grid = static_cast<unsigned>((groups + 7) / 8 * 8 * w.ty);
  // 512 threads: 8 waves over the pooling walk and both transforms (bench step +2.7 % over 256 at 128
  // images per GPU; profiles/r03_transform_threads_*)
  if (w.m == 4)
    pool_wino_in_kernel<4, pg, 512>
        <<<grid, 512, 0, s>>>(c1, V, groups, H1, W1, w.C, w.Hq, w.Wq, q_lo, Hp, Wp, P, c1_lo, w.ty, w.tx);
  else
    pool_wino_in_kernel<3, pg, 512>
        <<<grid, 512, 0, s>>>(c1, V, groups, H1, W1, w.C, w.Hq, w.Wq, q_lo, Hp, Wp, P, c1_lo, w.ty, w.tx);
  return hipGetLastError();
}

hipError_t wino_window_merge_input(const WinoPlan& w, const float* window, const float* p1, int n_off, int ty1, int tx1,
                                   int q_lo, int Hp, int Wp, int P, float* V, hipStream_t s, int pg) {
  if ((pg != 32 && pg != 16) || w.C % pg || w.Wq > kMaxWq || static_cast<long>(w.P) * w.C * npt(w.m) >= (1L << 31))
    return hipErrorInvalidValue;
  if (w.P == 0) return hipSuccess;
  const int groups = w.N * (w.C / pg);
  const unsigned grid = static_cast<unsigned>((groups + 7) / 8 * 8 * w.ty);
  if (w.m == 4 && pg == 16)
    pool_wino_in_kernel<4, 16, 256, false, true><<<grid, 256, 0, s>>>(window, V, groups, 0, 0, w.C, w.Hq, w.Wq, q_lo, Hp,
                                                                      Wp, P, 0, w.ty, w.tx, p1, n_off, ty1, tx1);
  else if (w.m == 4)
    pool_wino_in_kernel<4, 32, 512, false, true><<<grid, 512, 0, s>>>(window, V, groups, 0, 0, w.C, w.Hq, w.Wq, q_lo, Hp,
                                                                      Wp, P, 0, w.ty, w.tx, p1, n_off, ty1, tx1);
  else if (pg == 16)
    return hipErrorInvalidValue;
  else
    pool_wino_in_kernel<3, 32, 512, false, true><<<grid, 512, 0, s>>>(window, V, groups, 0, 0, w.C, w.Hq, w.Wq, q_lo, Hp,
                                                                      Wp, P, 0, w.ty, w.tx, p1, n_off, ty1, tx1);
  return hipGetLastError();
}

WinoPlan make_wino_plan(int N, int Hq, int Wq, int C, int K, int groups, int m) {
  if (m != 3 && m != 4) m = 3;
  WinoPlan w{};
  w.m = m;
  w.N = N;
  w.Hq = Hq;
  w.Wq = Wq;
  w.C = C;
  w.K = K;
  w.groups = groups;
  w.Ho = Hq - (wino::kR - 1);
  w.Wo = Wq - (wino::kR - 1);
  w.ty = (w.Ho + m - 1) / m;
  w.tx = (w.Wo + m - 1) / m;
  w.P = N * w.ty * w.tx;
  return w;
}

bool wino_eligible(int F, int S, int C, int K, int groups, int m) {
  // the fused GEMMs' configurations: F(3,5) 96 or 48 channels per group and filters per group a multiple
  // of 64; F(4,5) one group of 96 channels and a multiple of 64 filters (its workgroup tile is 64 filters)
  if (F != wino::kR || S != 1 || groups < 1 || C % groups || K % groups) return false;
  const int Cg = C / groups, Kg = K / groups;
  if (m == 4) return groups == 1 && C == 96 && K % 64 == 0;
  return (Cg == 96 || Cg == 48) && Kg % 64 == 0;
}

size_t wino_v_floats(const WinoPlan& w) { return static_cast<size_t>(w.P) * npt(w.m) * w.C; }
size_t wino_u_floats(const WinoPlan& w) { return static_cast<size_t>(npt(w.m)) * w.K * (w.C / w.groups); }

template <int M>
static void transform_weights(const WinoPlan& w, const float* w_kcff, std::vector<float>& u_kcff) {
  using T = WT<M>;
  constexpr int kN = T::kN;
  const int Cg = w.C / w.groups, Kg = w.K / w.groups, R = wino::kR;
  u_kcff.assign(wino_u_floats(w), 0.f);
  for (int g = 0; g < w.groups; ++g)
    for (int k = 0; k < Kg; ++k)
      for (int c = 0; c < Cg; ++c) {
        const float* f = w_kcff + ((static_cast<size_t>(g * Kg + k) * Cg + c) * R) * R;
        double tmp[kN][wino::kR];
        for (int a = 0; a < kN; ++a)
          for (int v = 0; v < R; ++v) {
            double s = 0;
            for (int u = 0; u < R; ++u) s += T::g(a, u) * f[u * R + v];
            tmp[a][v] = s;
          }
        for (int a = 0; a < kN; ++a)
          for (int b = 0; b < kN; ++b) {
            double s = 0;
            for (int v = 0; v < R; ++v) s += tmp[a][v] * T::g(b, v);
            const int ab = a * kN + b;
            u_kcff[(static_cast<size_t>(ab * w.groups + g) * Kg + k) * Cg + c] = static_cast<float>(s);
          }
      }
}

void wino_transform_weights_host(const WinoPlan& w, const float* w_kcff, std::vector<float>& u_kcff) {
  // U[(ab*groups + g)*Kg + k][c] = (G g_{k,c} G^T)[a][b], computed in fp64 then rounded once.
  if (w.m == 4)
    transform_weights<4>(w, w_kcff, u_kcff);
  else
    transform_weights<3>(w, w_kcff, u_kcff);
}

hipError_t wino_input(const WinoPlan& w, const float* x, float* V, hipStream_t s) {
  const long n = static_cast<long>(w.P) * w.C;
  if (n >= (1L << 31) || w.C % 2) return hipErrorInvalidValue;
  if (w.C % 32 == 0 && w.Wq <= kMaxWq && n * npt(w.m) < (1L << 31)) {  // band form (bit-identical V)
    if (w.P == 0) return hipSuccess;
    const int groups = w.N * (w.C / 32);
    const unsigned grid = static_cast<unsigned>((groups + 7) / 8 * 8 * w.ty);
    if (w.m == 4)
      pool_wino_in_kernel<4, 32, 512, false>
          <<<grid, 512, 0, s>>>(x, V, groups, 0, 0, w.C, w.Hq, w.Wq, 0, 0, 0, 0, 0, w.ty, w.tx);
    else
      pool_wino_in_kernel<3, 32, 512, false>
          <<<grid, 512, 0, s>>>(x, V, groups, 0, 0, w.C, w.Hq, w.Wq, 0, 0, 0, 0, 0, w.ty, w.tx);
    return hipGetLastError();
  }
  const long g = (n / 2 + kT - 1) / kT;
  const unsigned gg = static_cast<unsigned>(g < (1 << 20) ? g : (1 << 20));
  if (w.m == 4)
    wino_in2_kernel<4><<<gg, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
  else
    wino_in2_kernel<3><<<gg, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
  return hipGetLastError();
}

hipError_t wino_conv2(const WinoPlan& w, const float* V, const float* U, const float* bias, OutView out, bool relu,
                      hipStream_t s, const Knobs& k) {
  if (w.m == 4)
    return wino_gemm_conv2_f45(V, U, bias, out, w.P, w.ty, w.tx, w.Ho, w.Wo, w.K, relu, s, k.conv2_occ,
                               k.conv2_sched ? kConv2SchedAbl : 0);
  return wino_gemm_conv2(V, U, bias, out, w.P, w.ty, w.tx, w.Ho, w.Wo, w.C, w.K, w.groups, relu, s, k.conv2_occ);
}

}  // namespace anx::hip
