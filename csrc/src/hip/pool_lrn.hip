// Max-pool and fused max-pool + LRN for NHWC activations.
//
// Parity: poolKernel / lrnKernel (v3_cuda_only/src/layers_cuda.cu:78-152,
// v4_mpi_cuda/src/layers_mpi_cuda.cu:54-89). The reference runs pool2 and LRN2 as two kernels
// with a full HBM round trip in between and one thread per element; here pool2 + LRN is one
// pass: pooled pixels are staged in LDS and the cross-channel window is read from LDS.
// Both kernels move float4 (16 B/lane) per access; the pool writes through an OutView so pool1
// lands directly inside conv2's zero-bordered input buffer (no pad kernel, no copy).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>

#include "anx/lrn_math.hpp"
#include "anx/ops.hpp"

namespace anx::hip {
namespace {

constexpr int kThreads = 256;
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 max4(f32x4 a, f32x4 b) {
  return f32x4{fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w)};
}

// Max of an F x F window of float4 channel groups; `p` points at the window origin. For unpadded
// pooling every window of a valid output lies inside the input ((Ho-1)*S + F <= H), so the fixed-F
// path needs no bounds checks and issues all F*F loads back to back.
template <int F>
__device__ __forceinline__ f32x4 window_max(const float* p, int W, int C) {
  f32x4 v[F * F];
#pragma unroll
  for (int fh = 0; fh < F; ++fh)
#pragma unroll
    for (int fw = 0; fw < F; ++fw) v[fh * F + fw] = *reinterpret_cast<const f32x4*>(p + (fh * W + fw) * C);
  f32x4 m = v[0];
#pragma unroll
  for (int i = 1; i < F * F; ++i) m = max4(m, v[i]);
  return m;
}

// 32-bit index math (the 64-bit divisions of the generic kernel cost more than the loads).
template <int F, int S>
__global__ void __launch_bounds__(kThreads) maxpool_fixed_kernel(const float* __restrict__ x, int total, int H, int W,
                                                                 int C, int Ho, int Wo, OutView o) {
  const int C4 = C >> 2;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < total; i += gridDim.x * kThreads) {
    const int c4 = i % C4;
    int r = i / C4;
    const int ox = r % Wo;
    r /= Wo;
    const int oy = r % Ho;
    const int n = r / Ho;
    const f32x4 m = window_max<F>(x + nhwc(n, oy * S, ox * S, c4 * 4, H, W, C), W, C);
    float* dst = o.base + (static_cast<size_t>(n * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) * o.Cb + o.c_off +
                 c4 * 4;
    *reinterpret_cast<f32x4*>(dst) = m;
  }
}

__global__ void __launch_bounds__(kThreads) maxpool_vec4_kernel(const float* __restrict__ x, int N, int H, int W,
                                                                int C, int F, int S, int Ho, int Wo, OutView o) {
  const int C4 = C / 4;
  const size_t total = static_cast<size_t>(N) * Ho * Wo * C4;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int c4 = static_cast<int>(i % C4);
    size_t r = i / C4;
    const int ox = static_cast<int>(r % Wo);
    r /= Wo;
    const int oy = static_cast<int>(r % Ho);
    const int n = static_cast<int>(r / Ho);
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int fh = 0; fh < F; ++fh) {
      const int iy = oy * S + fh;
      if (iy >= H) break;
      const float* row = x + nhwc(n, iy, 0, c4 * 4, H, W, C);
      for (int fw = 0; fw < F; ++fw) {
        const int ix = ox * S + fw;
        if (ix >= W) break;
        m = max4(m, *reinterpret_cast<const f32x4*>(row + static_cast<size_t>(ix) * C));
      }
    }
    float* dst = o.base + (static_cast<size_t>(n * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) * o.Cb + o.c_off +
                 c4 * 4;
    *reinterpret_cast<f32x4*>(dst) = m;
  }
}

// One workgroup = PP output pixels x all C channels. Pass 1 pools into LDS, pass 2 applies LRN.
// FF > 0: compile-time window (no bounds checks, loads issued together); FF == 0: runtime F.
template <int FF>
__global__ void __launch_bounds__(kThreads) maxpool_lrn_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int N, int H, int W, int C, int F, int S, int Ho,
                                                               int Wo, int PP, int size, float a, float beta,
                                                               float k) {
  extern __shared__ __attribute__((aligned(16))) float pooled[];  // [PP][C]
  const int C4 = C / 4;
  const int P = N * Ho * Wo;  // < 2^31 (checked by the launcher)
  const int p0 = blockIdx.x * PP;
  const int chunks = PP * C4;
  for (int t = threadIdx.x; t < chunks; t += blockDim.x) {
    const int pl = t / C4, c4 = t - pl * C4;
    const int p = p0 + pl;
    f32x4 m = {0.f, 0.f, 0.f, 0.f};
    if (p < P) {
      const int ox = p % Wo;
      const int r = p / Wo;
      const int oy = r % Ho;
      const int n = r / Ho;
      if constexpr (FF > 0) {
        *reinterpret_cast<f32x4*>(pooled + pl * C + c4 * 4) = window_max<FF>(x + nhwc(n, oy * S, ox * S, c4 * 4, H, W, C), W, C);
        continue;
      }
      m = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      for (int fh = 0; fh < F; ++fh) {
        const int iy = oy * S + fh;
        if (iy >= H) break;
        const float* row = x + nhwc(n, iy, 0, c4 * 4, H, W, C);
        for (int fw = 0; fw < F; ++fw) {
          const int ix = ox * S + fw;
          if (ix >= W) break;
          m = max4(m, *reinterpret_cast<const f32x4*>(row + static_cast<size_t>(ix) * C));
        }
      }
    }
    *reinterpret_cast<f32x4*>(pooled + pl * C + c4 * 4) = m;
  }
  __syncthreads();
  const int half = size / 2;
  for (int t = threadIdx.x; t < chunks; t += blockDim.x) {
    const int pl = t / C4, c4 = t - pl * C4;
    const int p = p0 + pl;
    if (p >= P) continue;
    const float* row = pooled + pl * C;
    const int c0 = c4 * 4;
    f32x4 out;
    if (half == 2) {
      // AlexNet's size-5 window: one ds_read_b128 for the own 4 channels and two ds_read_b64 for
      // the 2 neighbours on each side (lane-contiguous, conflict-free; 20 strided ds_read_b32
      // per thread were 4-way bank conflicted). Channels outside [0, C) contribute fmaf(0,0,s)
      // = s, so the sums are bitwise those of the clamped loop below.
      using f32x2 = __attribute__((ext_vector_type(2))) float;
      const f32x4 own = *reinterpret_cast<const f32x4*>(row + c0);
      const f32x2 lft = c0 >= 2 ? *reinterpret_cast<const f32x2*>(row + c0 - 2) : f32x2{0.f, 0.f};
      const f32x2 rgt = c0 + 4 < C ? *reinterpret_cast<const f32x2*>(row + c0 + 4) : f32x2{0.f, 0.f};
      const float w[8] = {lft.x, lft.y, own.x, own.y, own.z, own.w, rgt.x, rgt.y};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float s = 0.f;
#pragma unroll
        for (int u = e; u < e + 5; ++u) s = fmaf(w[u], w[u], s);
        out[e] = w[e + 2] * lrn_scale(s, k, a, beta);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + e;
        const int lo = c - half < 0 ? 0 : c - half;
        const int hi = c + half >= C ? C - 1 : c + half;
        float s = 0.f;
        for (int j = lo; j <= hi; ++j) s = fmaf(row[j], row[j], s);
        out[e] = row[c] * lrn_scale(s, k, a, beta);
      }
    }
    *reinterpret_cast<f32x4*>(y + static_cast<size_t>(p) * C + c4 * 4) = out;
  }
}

// Pool2 + LRN for C = 256 (AlexNet): a wave owns a pooled pixel per step, lane i channels
// 4i..4i+3, and takes U consecutive pixels per step with all 9U window loads in flight (U = 1 was
// latency-bound at 3.7 TB/s). The 9 loads of a lane are 16 B each and a wave's loads are whole
// 1-KiB pixel rows; the LRN neighbours (channels 4i-2, 4i-1, 4i+4, 4i+5) come from lanes i-1 / i+1
// by ds_bpermute, so there is no LDS tile, no barrier, and no bank conflicts. The squared-sum order
// is that of maxpool_lrn_kernel (left to right), so both kernels give bitwise equal results.
// MERGE: x is a pooled map [N][Ho][Wo][256] from the pool2 GEMM epilogue (wino_gemm_conv2_f45_pool), p2 the
// upper workgroups' partial maxima of the straddling windows (pool2_straddles of image n % sub, ty2 x tx2
// tiles per image): the pooled pixel is max(x, p2) there, x elsewhere.
template <int F, int U, bool MERGE = false>
__global__ void __launch_bounds__(kThreads) maxpool_lrn256_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                  int P, int H, int W, int S, int Ho, int Wo, float a,
                                                                  float beta, float k, const float* __restrict__ p2 = nullptr,
                                                                  int ty2 = 0, int tx2 = 0, int sub = 1) {
  constexpr int C = 256;
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (kThreads / 64);
  for (int base = (blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * U; base < P; base += nw * U) {  // wave-uniform
    f32x4 own[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = base + u;
      if (p < P) {
        const int ox = p % Wo, r = p / Wo, oy = r % Ho, n = r / Ho;
        if constexpr (MERGE) {
          own[u] = *reinterpret_cast<const f32x4*>(x + static_cast<size_t>(p) * C + lane * 4);
          if (pool2_straddles(n % sub, oy, ox, ty2, tx2)) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(p2 + static_cast<size_t>(p) * C + lane * 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) own[u][i] = fmaxf(own[u][i], q[i]);
          }
        } else {
          own[u] = window_max<F>(x + nhwc(n, oy * S, ox * S, lane * 4, H, W, C), W, C);
        }
      } else {
        own[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // neighbours: left pair = (z, w) of lane-1, right pair = (x, y) of lane+1; zero past the edges
    const int left = ((lane + 63) & 63) * 4, right = ((lane + 1) & 63) * 4;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float l0 = __int_as_float(__builtin_amdgcn_ds_bpermute(left, __float_as_int(own[u].z)));
      float l1 = __int_as_float(__builtin_amdgcn_ds_bpermute(left, __float_as_int(own[u].w)));
      float r0 = __int_as_float(__builtin_amdgcn_ds_bpermute(right, __float_as_int(own[u].x)));
      float r1 = __int_as_float(__builtin_amdgcn_ds_bpermute(right, __float_as_int(own[u].y)));
      if (lane == 0) l0 = l1 = 0.f;
      if (lane == 63) r0 = r1 = 0.f;
      const int p = base + u;
      if (p >= P) continue;
      const float w[8] = {l0, l1, own[u].x, own[u].y, own[u].z, own[u].w, r0, r1};
      f32x4 out;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sq = 0.f;
#pragma unroll
        for (int t = e; t < e + 5; ++t) sq = fmaf(w[t], w[t], sq);
        out[e] = w[e + 2] * lrn_scale(sq, k, a, beta);
      }
      *reinterpret_cast<f32x4*>(y + static_cast<size_t>(p) * C + lane * 4) = out;
    }
  }
}

}  // namespace

hipError_t lrn_pooled_merge(const float* pooled, const float* p2, float* y, int N, int Hp, int Wp, int C, int ty2,
                            int tx2, int sub, int size, float alpha, float beta, float k, LrnMode mode, hipStream_t s,
                            int max_wgs) {
  const long P = static_cast<long>(N) * Hp * Wp;
  if (P == 0) return hipSuccess;
  if (C != 256 || size != 5 || sub < 1 || P * C >= (1L << 31)) return hipErrorInvalidValue;
  const float a = mode == LrnMode::DivN ? alpha / static_cast<float>(size) : alpha;
  constexpr int U = 2;  // pixels per wave step (as maxpool_lrn)
  const long waves = (P + U - 1) / U;
  unsigned g = static_cast<unsigned>((waves + kThreads / 64 - 1) / (kThreads / 64));
  if (max_wgs > 0 && g > static_cast<unsigned>(max_wgs)) g = static_cast<unsigned>(max_wgs);  // the waves walk the rest
  maxpool_lrn256_kernel<3, U, true><<<g, kThreads, 0, s>>>(pooled, y, static_cast<int>(P), Hp, Wp, 1, Hp, Wp, a, beta,
                                                           k, p2, ty2, tx2, sub);
  return hipGetLastError();
}

hipError_t maxpool(const float* x, int N, int H, int W, int C, int F, int S, OutView out, hipStream_t s) {
  const int Ho = pool_out_dim(H, F, S), Wo = pool_out_dim(W, F, S);
  const size_t total = static_cast<size_t>(N) * Ho * Wo * (C / 4);
  if (total == 0) return hipSuccess;
  if (C % 4 || out.Cb % 4 || out.c_off % 4) return hipErrorInvalidValue;
  if (F == 3 && S == 2 && total < (1UL << 31)) {
    const unsigned g = static_cast<unsigned>(std::min<size_t>((total + kThreads - 1) / kThreads, 1 << 20));
    maxpool_fixed_kernel<3, 2><<<g, kThreads, 0, s>>>(x, static_cast<int>(total), H, W, C, Ho, Wo, out);
    return hipGetLastError();
  }
  size_t g = (total + kThreads - 1) / kThreads;
  if (g > 65535) g = 65535;
  maxpool_vec4_kernel<<<static_cast<unsigned>(g), kThreads, 0, s>>>(x, N, H, W, C, F, S, Ho, Wo, out);
  return hipGetLastError();
}

hipError_t maxpool_lrn(const float* x, float* y, int N, int H, int W, int C, int F, int S, int size, float alpha,
                       float beta, float k, LrnMode mode, hipStream_t s) {
  const int Ho = pool_out_dim(H, F, S), Wo = pool_out_dim(W, F, S);
  const long P = static_cast<long>(N) * Ho * Wo;
  if (P == 0) return hipSuccess;
  if (C % 4 || C > 8192 || P >= (1L << 31)) return hipErrorInvalidValue;
  const int PP = C >= 4096 ? 1 : 4096 / C;  // 16 KB of LDS per workgroup
  const long blocks = (P + PP - 1) / PP;
  const float a = mode == LrnMode::DivN ? alpha / static_cast<float>(size) : alpha;
  if (F == 3 && C == 256 && size == 5) {
    constexpr int U = 2;  // pixels per wave step
    const long waves = (P + U - 1) / U;
    const unsigned g = static_cast<unsigned>((waves + kThreads / 64 - 1) / (kThreads / 64));
    maxpool_lrn256_kernel<3, U><<<g, kThreads, 0, s>>>(x, y, static_cast<int>(P), H, W, S, Ho, Wo, a, beta, k);
    return hipGetLastError();
  }
  if (F == 3)
    maxpool_lrn_kernel<3><<<static_cast<unsigned>(blocks), kThreads, PP * C * sizeof(float), s>>>(
        x, y, N, H, W, C, F, S, Ho, Wo, PP, size, a, beta, k);
  else
    maxpool_lrn_kernel<0><<<static_cast<unsigned>(blocks), kThreads, PP * C * sizeof(float), s>>>(
        x, y, N, H, W, C, F, S, Ho, Wo, PP, size, a, beta, k);
  return hipGetLastError();
}

}  // namespace anx::hip
