// Winograd F(3x3, 5x5) convolution for stride-1 5x5 layers (AlexNet Conv2), fp32 end to end.
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

namespace anx::hip {
namespace {

using f32x2 = __attribute__((ext_vector_type(2))) float;
constexpr int kT = 256;
constexpr int kN = wino::kN, kM = wino::kM;

// Thread = (tile, 2 channels): consecutive threads read consecutive channel pairs (coalesced NHWC
// 8-B loads and stores); the 7x7 patch streams through t = B^T d one input row at a time. 98
// transform registers keep 3+ waves per SIMD. C even.
__global__ void __launch_bounds__(kT) wino_in2_kernel(const float* __restrict__ x, float* __restrict__ V, int N, int Hq,
                                                      int Wq, int C, int ty, int tx) {
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
        if (wino::kBT[a][u] != 0.f)
#pragma unroll
          for (int v = 0; v < kN; ++v) {  // per-component fmaf (no packed FMA): the transform's rounding
            t[a][v].x = fmaf(wino::kBT[a][u], row[v].x, t[a][v].x);
            t[a][v].y = fmaf(wino::kBT[a][u], row[v].y, t[a][v].y);
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
          if (wino::kBT[b][v] != 0.f) {
            s2.x = fmaf(wino::kBT[b][v], t[a][v].x, s2.x);
            s2.y = fmaf(wino::kBT[b][v], t[a][v].y, s2.y);
          }
        *reinterpret_cast<f32x2*>(out + static_cast<size_t>(a * kN + b) * C) = s2;
      }
  }
}

}  // namespace

WinoPlan make_wino_plan(int N, int Hq, int Wq, int C, int K, int groups) {
  WinoPlan w{};
  w.N = N;
  w.Hq = Hq;
  w.Wq = Wq;
  w.C = C;
  w.K = K;
  w.groups = groups;
  w.Ho = Hq - (wino::kR - 1);
  w.Wo = Wq - (wino::kR - 1);
  w.ty = (w.Ho + kM - 1) / kM;
  w.tx = (w.Wo + kM - 1) / kM;
  w.P = N * w.ty * w.tx;
  return w;
}

bool wino_eligible(int F, int S, int C, int K, int groups) {
  // the fused GEMM's configurations: 96 or 48 channels per group, filters per group a multiple of 64
  if (F != wino::kR || S != 1 || groups < 1 || C % groups || K % groups) return false;
  const int Cg = C / groups, Kg = K / groups;
  return (Cg == 96 || Cg == 48) && Kg % 64 == 0;
}

size_t wino_v_floats(const WinoPlan& w) { return static_cast<size_t>(w.P) * kN * kN * w.C; }
size_t wino_u_floats(const WinoPlan& w) { return static_cast<size_t>(kN * kN) * w.K * (w.C / w.groups); }

void wino_transform_weights_host(const WinoPlan& w, const float* w_kcff, std::vector<float>& u_kcff) {
  // U[(ab*groups + g)*Kg + k][c] = (G g_{k,c} G^T)[a][b], computed in fp64 then rounded once.
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
            for (int u = 0; u < R; ++u) s += wino::kG[a][u] * f[u * R + v];
            tmp[a][v] = s;
          }
        for (int a = 0; a < kN; ++a)
          for (int b = 0; b < kN; ++b) {
            double s = 0;
            for (int v = 0; v < R; ++v) s += tmp[a][v] * wino::kG[b][v];
            const int ab = a * kN + b;
            u_kcff[(static_cast<size_t>(ab * w.groups + g) * Kg + k) * Cg + c] = static_cast<float>(s);
          }
      }
}

hipError_t wino_input(const WinoPlan& w, const float* x, float* V, hipStream_t s) {
  const long n = static_cast<long>(w.P) * w.C;
  if (n >= (1L << 31) || w.C % 2) return hipErrorInvalidValue;
  const long g = (n / 2 + kT - 1) / kT;
  const unsigned gg = static_cast<unsigned>(g < (1 << 20) ? g : (1 << 20));
  wino_in2_kernel<<<gg, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
  return hipGetLastError();
}

hipError_t wino_conv2(const WinoPlan& w, const float* V, const float* U, const float* bias, OutView out, bool relu,
                      hipStream_t s, const Knobs& k) {
  return wino_gemm_conv2(V, U, bias, out, w.P, w.ty, w.tx, w.Ho, w.Wo, w.C, w.K, w.groups, relu, s, k.conv2_occ);
}

}  // namespace anx::hip
