// Conv1 (11x11, stride 4, C = 3, no padding) as Winograd F(3x3,3x3) on the polyphase image.
//
// Polyphase rewrite (space-to-depth by the stride; exact):
//   X'[n][i][j][ch]   = x[n][4i+rh][4j+rw][c],      ch = (rh*4 + rw)*3 + c    (48 channels)
//   W'[k][ch][qh][qw] = w[k][c][4qh+rh][4qw+rw]     (0 where 4qh+rh or 4qw+rw >= F)
//   conv1(x, w)[n][oy][ox][k] = sum_{qh,qw<3} sum_ch X'[n][oy+qh][ox+qw][ch] * W'[k][ch][qh][qw]
// i.e. a stride-1 3x3 convolution over 48 channels. F(3x3,3x3) produces a 3x3 output tile with 25
// multiplies per (channel, filter) instead of 81, so Conv1's matrix-core work drops from 416 MACs
// per output (the direct implicit GEMM's taps4-padded K, conv_mfma.hip) to 25*48/9 = 133.
// The reference computes Conv1 one output per thread with no reuse (convKernel,
// v3_cuda_only/src/layers_cuda.cu:20-46; v4_mpi_cuda/src/layers_mpi_cuda.cu:25-47).
//
// Two launches on the caller's stream:
//   1. conv1_wino_in_kernel : image rows -> V [P][25][48] (P = N*ty*tx tiles; VALU, 16-B loads)
//   2. the fused Winograd GEMM (wino_gemm.hpp, 64 tiles x 32 filters per workgroup: Conv1's 96
//      filters are exactly 3 workgroup columns): M_ab = V_ab . U_ab on v_mfma_f32_32x32x2_f32
//      (exact fp32), folded into the 3x3 outputs in registers, bias + ReLU + NHWC store through an
//      OutView.
// Numerics: tests/test_winograd_math.py checks the algebra in fp64; the fp32 error of the point set
// is ~1e-7 of sum|terms| (tools/winograd_numerics.py).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

#include "anx/ops.hpp"
#include "anx/winograd_f33.hpp"

namespace anx::hip {
namespace {

namespace w33 = anx::wino33;
using f32x4 = __attribute__((ext_vector_type(4))) float;
// 12-float (rw, c) runs start at any float of an image row: 4-byte aligned 16-B loads (ROCm runs
// gfx9 in unaligned-access mode; still one global_load_dwordx4).
using f32x4u = __attribute__((ext_vector_type(4), aligned(4))) float;

constexpr int kT = 256;
constexpr int kPh = 4;                     // conv1 stride = polyphase factor
constexpr int kCh = kPh * kPh * 3;         // 48 polyphase channels
constexpr int kN5 = w33::kN;               // 5x5 transform tile
constexpr int kPts = kN5 * kN5;            // 25 transform points
constexpr int kPitch = w33::kM * kPh;      // 12 image rows/cols between tile origins
constexpr int kBN = 32;                    // filters per GEMM workgroup column

// ---------------------------------------------------------------------------------------------
// Input transform. Thread = (tile p, phase row rh, 16-B unit j): at each of the 5x5 X' positions
// of the tile the 12 floats (rw, c) of phase row rh are 3 contiguous float4 units of one image row.
// Consecutive threads cover consecutive channels, so V rows (48 floats per (p, ab)) are written
// as whole 192-B runs.
__global__ void __launch_bounds__(kT) conv1_wino_in_kernel(const float* __restrict__ x, float* __restrict__ V,
                                                           int total, int Hin, int rowf, int ty, int tx) {
  for (int i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    const int q = i % 12;
    const int p = i / 12;
    const int rh = q / 3, j = q - rh * 3;
    const int tj = p % tx;
    const int pq = p / tx;
    const int ti = pq % ty;
    const int n = pq / ty;
    const float* img = x + static_cast<size_t>(n) * Hin * rowf;
    f32x4 t[kN5][kN5];  // t = B^T d, one input row u at a time
#pragma unroll
    for (int a = 0; a < kN5; ++a)
#pragma unroll
      for (int v = 0; v < kN5; ++v) t[a][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < kN5; ++u) {
      const int row = ti * kPitch + kPh * u + rh;
      f32x4 d[kN5];
#pragma unroll
      for (int v = 0; v < kN5; ++v) {
        const int o = (tj * kPitch + kPh * v) * 3 + 4 * j;  // float offset inside the image row
        d[v] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (row < Hin) {
          const float* src = img + static_cast<size_t>(row) * rowf + o;
          if (o + 4 <= rowf) {
            d[v] = *reinterpret_cast<const f32x4u*>(src);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (o + e < rowf) d[v][e] = src[e];
          }
        }
      }
#pragma unroll
      for (int a = 0; a < kN5; ++a)
        if (w33::kBT[a][u] != 0.f)
#pragma unroll
          for (int v = 0; v < kN5; ++v) t[a][v] += w33::kBT[a][u] * d[v];
    }
    float* out = V + static_cast<size_t>(p) * kPts * kCh + rh * 12 + 4 * j;
#pragma unroll
    for (int a = 0; a < kN5; ++a)
#pragma unroll
      for (int b = 0; b < kN5; ++b) {
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int v = 0; v < kN5; ++v)
          if (w33::kBT[b][v] != 0.f) s += w33::kBT[b][v] * t[a][v];
        *reinterpret_cast<f32x4*>(out + (a * kN5 + b) * kCh) = s;
      }
  }
}

// Band form of the input transform: one workgroup = (image, tile row, NRH of the 4 phase rows, NCS
// column splits). The tile row's image rows of those phases (5 polyphase rows x NRH) are copied to LDS
// with 16-B loads (each image row read once per tile row, not once per tile it touches), B^T runs down
// each (phase row, float column) in place, then B along each tile's 5 polyphase columns. Same fmaf
// expressions in the same order as conv1_wino_in_kernel, so V is bit-identical. The launcher's default
// (Knobs::conv1_band = 2) is NRH = 4 x NCS = 2: all 4 phase rows of half the tile columns, 30 KiB of
// LDS, each 192-B V segment written whole (profiles/r03_band_split_*). conv1_band = 1 keeps NRH = 2 x
// NCS = 1 (27 KiB). All 4 phase rows of a whole tile row (54 KiB) rarely fit beside a CU's Winograd
// GEMM workgroups under stream lanes (236 k vs 244 k images/s, profiles/r03_conv1_band2_*); one phase
// row (14 KiB) adds more workgroups than co-residency gains (profiles/r03_transform_lds_*).
constexpr int kMaxRowF = 684;  // LDS row stride (floats, 16-B multiple): image width <= 228
constexpr int kMaxSplitF = 384;  // column-split rows: <= 10 tiles per split (36 * 10 + 24 floats)
template <int NRH, int NCS, int NT>  // phase rows, column splits, threads per workgroup
__global__ void __launch_bounds__(NT) conv1_wino_band_kernel(const float* __restrict__ x, float* __restrict__ V, int N,
                                                             int Hin, int rowf, int ty, int tx) {
  constexpr int RG = kPh / NRH, BR = kN5 * NRH;  // phase-row groups per tile row, LDS rows
  constexpr int MAXF = NCS == 1 ? kMaxRowF : kMaxSplitF;
  __shared__ __attribute__((aligned(16))) float band[BR * MAXF];
  const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
  const int n = (j / (ty * RG * NCS)) * 8 + xcd, rem = j % (ty * RG * NCS);
  const int ti = rem / (RG * NCS), rg = (rem / NCS) % RG, cs = rem % NCS;
  if (n >= N) return;  // whole workgroup, before any barrier
  // this split's tiles [tj0, tj1) read image floats [f0, f0 + width) of each row (zero past the image)
  const int tps = (tx + NCS - 1) / NCS, tj0 = cs * tps, tj1 = min(tx, tj0 + tps);
  const int f0 = tj0 * kPitch * 3;
  const int rowp = NCS == 1 ? (rowf + 3) & ~3 : (tps * kPitch + 2 * kPh) * 3;
  const int tid = threadIdx.x;
  const float* img = x + static_cast<size_t>(n) * Hin * rowf + f0;
  // 1. LDS row u*NRH + rl = image row ti*12 + 4u + rg*NRH + rl (zero past the image)
  const int u4 = rowp / 4;
  for (int it = tid; it < BR * u4; it += NT) {
    const int lr = it / u4, k = (it - lr * u4) * 4;
    const int row = ti * kPitch + kPh * (lr / NRH) + rg * NRH + lr % NRH;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < Hin) {
      const float* p = img + static_cast<size_t>(row) * rowf + k;
      if (f0 + k + 4 <= rowf) {
        v = *reinterpret_cast<const f32x4u*>(p);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (f0 + k + e < rowf) v[e] = p[e];
      }
    }
    *reinterpret_cast<f32x4*>(&band[lr * rowp + k]) = v;
  }
  __syncthreads();
  // 2. t = B^T d over the 5 polyphase rows of each (phase row, float column), in place
  for (int it = tid; it < NRH * rowp; it += NT) {
    const int f = it % rowp, rl = it / rowp;
    float d[kN5], t[kN5];
#pragma unroll
    for (int u = 0; u < kN5; ++u) d[u] = band[(u * NRH + rl) * rowp + f];
#pragma unroll
    for (int a = 0; a < kN5; ++a) {
      t[a] = 0.f;
#pragma unroll
      for (int u = 0; u < kN5; ++u)
        if (w33::kBT[a][u] != 0.f) t[a] += w33::kBT[a][u] * d[u];
    }
#pragma unroll
    for (int a = 0; a < kN5; ++a) band[(a * NRH + rl) * rowp + f] = t[a];
  }
  __syncthreads();
  // 3. V[p][a*5 + b][rh*12 + 4jq .. +3] = sum_v B^T[b][v] t[a][v]: one (tile, a, 16-B channel unit) per
  // thread; the unit's 4 channels are 4 consecutive floats of the image row (rw, c)
  for (int it = tid; it < (tj1 - tj0) * kN5 * 3 * NRH; it += NT) {
    const int q = it % (3 * NRH), rest = it / (3 * NRH), a = rest % kN5, tj = tj0 + rest / kN5;
    const int rl = q / 3, jq = q - rl * 3, rh = rg * NRH + rl;
    const float* row = band + (a * NRH + rl) * rowp;
    f32x4 t[kN5];
#pragma unroll
    for (int v = 0; v < kN5; ++v) {
      const int o = ((tj - tj0) * kPitch + kPh * v) * 3 + 4 * jq;
      t[v] = o < rowp ? *reinterpret_cast<const f32x4*>(row + o) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int p = (n * ty + ti) * tx + tj;
    float* out = V + static_cast<size_t>(p) * kPts * kCh + a * kN5 * kCh + rh * 12 + 4 * jq;
#pragma unroll
    for (int bb = 0; bb < kN5; ++bb) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < kN5; ++v)
        if (w33::kBT[bb][v] != 0.f) s += w33::kBT[bb][v] * t[v];
      *reinterpret_cast<f32x4*>(out + bb * kCh) = s;
    }
  }
}

}  // namespace

bool conv1_wino_eligible(int C, int K, int F, int S, int P, int groups) {
  // ceil(F/4) == 3 taps per phase axis; 3 input channels -> 48 polyphase channels
  return C == 3 && S == kPh && P == 0 && groups == 1 && F > 2 * kPh && F <= 3 * kPh && K > 0 && K % kBN == 0;
}

Conv1WinoPlan make_conv1_wino_plan(int N, int Hin, int W, int K, int F) {
  Conv1WinoPlan w{};
  w.N = N;
  w.Hin = Hin;
  w.W = W;
  w.K = K;
  w.F = F;
  w.H1 = conv_out_dim(Hin, F, kPh, 0);
  w.W1 = conv_out_dim(W, F, kPh, 0);
  w.ty = (w.H1 + 2) / 3;
  w.tx = (w.W1 + 2) / 3;
  w.P = N * w.ty * w.tx;
  return w;
}

size_t conv1_wino_v_floats(const Conv1WinoPlan& w) { return static_cast<size_t>(w.P) * kPts * kCh; }
size_t conv1_wino_u_floats(int K) { return static_cast<size_t>(kPts) * K * kCh; }

void conv1_wino_weights_host(int K, int F, const float* w_kcff, std::vector<float>& u) {
  // U[ab][k][ch] = (G W'_{k,ch} G^T)[a][b], fp64 then rounded once
  u.assign(conv1_wino_u_floats(K), 0.f);
  for (int k = 0; k < K; ++k)
    for (int ch = 0; ch < kCh; ++ch) {
      const int rh = ch / 12, rw = (ch % 12) / 3, c = ch % 3;
      double g[3][3];
      for (int qh = 0; qh < 3; ++qh)
        for (int qw = 0; qw < 3; ++qw) {
          const int fh = kPh * qh + rh, fw = kPh * qw + rw;
          g[qh][qw] = (fh < F && fw < F) ? w_kcff[((static_cast<size_t>(k) * 3 + c) * F + fh) * F + fw] : 0.0;
        }
      double tmp[kN5][3];
      for (int a = 0; a < kN5; ++a)
        for (int qw = 0; qw < 3; ++qw) {
          double s = 0;
          for (int qh = 0; qh < 3; ++qh) s += w33::kG[a][qh] * g[qh][qw];
          tmp[a][qw] = s;
        }
      for (int a = 0; a < kN5; ++a)
        for (int b = 0; b < kN5; ++b) {
          double s = 0;
          for (int qw = 0; qw < 3; ++qw) s += tmp[a][qw] * w33::kG[b][qw];
          u[(static_cast<size_t>(a * kN5 + b) * K + k) * kCh + ch] = static_cast<float>(s);
        }
    }
}

hipError_t conv1_wino(const Conv1WinoPlan& w, const float* x, float* V, const float* U, const float* bias, OutView out,
                      bool relu, hipStream_t s, const Knobs& kn) {
  if (w.P == 0 || w.H1 <= 0 || w.W1 <= 0) return hipSuccess;
  if (kn.conv1_fused && conv1_fused_eligible(w, out)) return conv1_fused(w, x, U, bias, out, relu, s);
  if (w.K % kBN || static_cast<long>(w.P) * kPts * kCh >= (1L << 31) || static_cast<long>(w.P) * 12 >= (1L << 31) ||
      out.Cb % 4 || out.c_off % 4)  // 16-B epilogue stores
    return hipErrorInvalidValue;
  if (kn.conv1_band && w.W * 3 <= kMaxRowF) {
    constexpr int kNRH = 2;  // phase rows per workgroup: 27 KiB of LDS (1 and 4 ran slower under lanes)
    const unsigned grid = static_cast<unsigned>((w.N + 7) / 8 * 8 * w.ty * (kPh / kNRH));
    if (kn.conv1_band == 2 && (w.tx + 1) / 2 * 36 + 24 <= kMaxSplitF) {  // all 4 phase rows, 2 column halves
      const unsigned g2 = static_cast<unsigned>((w.N + 7) / 8 * 8 * w.ty * 2);
      conv1_wino_band_kernel<4, 2, 512><<<g2, 512, 0, s>>>(x, V, w.N, w.Hin, w.W * 3, w.ty, w.tx);
    } else {
      conv1_wino_band_kernel<kNRH, 1, 512><<<grid, 512, 0, s>>>(x, V, w.N, w.Hin, w.W * 3, w.ty, w.tx);  // 8 waves
    }
  } else {
    const int total = w.P * 12;
    long g = (total + kT - 1) / kT;
    if (g > (1 << 20)) g = 1 << 20;
    conv1_wino_in_kernel<<<static_cast<unsigned>(g), kT, 0, s>>>(x, V, total, w.Hin, w.W * 3, w.ty, w.tx);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return wino_gemm_conv1(V, U, bias, out, w.P, w.ty, w.tx, w.H1, w.W1, w.K, relu, s, kn.conv1_occ);
}

}  // namespace anx::hip
