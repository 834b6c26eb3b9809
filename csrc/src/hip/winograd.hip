// Winograd F(3x3, 5x5) convolution for stride-1 5x5 layers (AlexNet Conv2), fp32 end to end.
//
//   Y = A^T [ U (.) V ] A,  U = G g G^T (49 x C x K, once per weight set, host fp64 -> fp32),
//                           V = B^T d B (per 7x7 input tile and channel), 3x3 outputs per tile.
// 49 multiplies per 9 outputs instead of 225: Conv2's 896 MFLOP/image become 195 MFLOP/image of
// MFMA work. The reference has no fast-convolution algorithm (direct loops everywhere:
// v3_cuda_only/src/layers_cuda.cu:20-46). fp32 error of this point set is ~5e-7 of sum|terms|
// (tools/winograd_numerics.py), the same order as the fp32 accumulation error of the direct sum.
//
// Three launches, all on the caller's stream:
//   1. input transform  : window [N][Hq][Wq][C] -> V [P][49][C]        (VALU, float4 over channels)
//   2. 49 batched GEMMs : V x U -> M [P][49][K]  = a grouped 1x1 conv on the MFMA implicit-GEMM
//                         kernel (conv_mfma.hip), groups = 49 * conv_groups
//   3. output transform : M -> Y = A^T M A + bias, ReLU, NHWC conv output (VALU, float4 over filters)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "anx/ops.hpp"
#include "anx/winograd_f35.hpp"

namespace anx::hip {
namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
constexpr int kT = 256;
constexpr int kN = wino::kN, kM = wino::kM;

// One thread per (tile, channel): consecutive threads read consecutive channels (coalesced NHWC),
// the 7x7 patch streams through t = B^T d one input row at a time (t: 49 registers).
template <bool NT>
__global__ void __launch_bounds__(kT) wino_in_kernel(const float* __restrict__ x, float* __restrict__ V, int N,
                                                     int Hq, int Wq, int C, int ty, int tx) {
  // 32-bit index math (total < 2^31, checked by the launcher): 64-bit divisions cost more than the loads
  const int total = N * ty * tx * C;
  for (int i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    const int c = i % C;
    const int p = i / C;
    const int tj = p % tx;
    const int q = p / tx;
    const int ti = q % ty;
    const int n = q / ty;
    float t[kN][kN];
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int v = 0; v < kN; ++v) t[a][v] = 0.f;
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int yy = ti * kM + u;
      float row[kN];
#pragma unroll
      for (int v = 0; v < kN; ++v) {
        const int xx = tj * kM + v;
        row[v] = (yy < Hq && xx < Wq) ? x[((static_cast<size_t>(n) * Hq + yy) * Wq + xx) * C + c] : 0.f;
      }
#pragma unroll
      for (int a = 0; a < kN; ++a)
        if (wino::kBT[a][u] != 0.f)
#pragma unroll
          for (int v = 0; v < kN; ++v) t[a][v] = fmaf(wino::kBT[a][u], row[v], t[a][v]);
    }
    // V = t B, stored [p][a*7+b][c]
    float* out = V + static_cast<size_t>(p) * (kN * kN) * C + c;
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int b = 0; b < kN; ++b) {
        float s2 = 0.f;
#pragma unroll
        for (int v = 0; v < kN; ++v)
          if (wino::kBT[b][v] != 0.f) s2 = fmaf(wino::kBT[b][v], t[a][v], s2);
        if constexpr (NT)
          __builtin_nontemporal_store(s2, out + static_cast<size_t>(a * kN + b) * C);
        else
          out[static_cast<size_t>(a * kN + b) * C] = s2;
      }
  }
}

// The same transform with 2 channels per thread (8-B loads and stores: half the memory instructions
// of the scalar kernel for the same bytes; 98 transform registers keep 3+ waves per SIMD). C even.
template <bool NT>
__global__ void __launch_bounds__(kT) wino_in2_kernel(const float* __restrict__ x, float* __restrict__ V, int N,
                                                      int Hq, int Wq, int C, int ty, int tx) {
  const int C2 = C >> 1;
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
          for (int v = 0; v < kN; ++v) {  // per-component fmaf: bit-identical to the scalar kernel
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
        if constexpr (NT)
          __builtin_nontemporal_store(s2, reinterpret_cast<f32x2*>(out + static_cast<size_t>(a * kN + b) * C));
        else
          *reinterpret_cast<f32x2*>(out + static_cast<size_t>(a * kN + b) * C) = s2;
      }
  }
}

struct WinoPoolArgs {
  int N, Hq, Wq, C, ty, tx;  // window / tile geometry (as wino_in_kernel)
  int H1, W1, Wp, pad;       // conv1 rows in the buffer, conv1 width, pool1 width, window border
  int q_lo, p1_lo, p1_hi, c1_lo;
};

// Pool1 fused into the input transform: the same V as maxpool(c1 -> zero-bordered window) followed
// by wino_in_kernel, without the window round trip through HBM (84 MB written + 111 MB read per
// 300 images) and one launch fewer. Window row r is pool1 row pr = r + q_lo (pool rows outside
// [p1_lo, p1_hi) and columns outside [0, Wp) are the zero border); pool1 row pr is the max over
// conv1 rows 2pr..2pr+2 (local rows 2pr - c1_lo ...) and columns 2px..2px+2. conv1 outputs are
// post-ReLU (>= 0) and a max is order-free, so V is bit-identical to the unfused pair.
// Workgroup = (image, tile row, 32 channels), 320 threads = 10 slots x 32 channels: phase 1 pools
// the tile row's 7 window rows x Wq columns into LDS (one thread per column walks the 15 conv1
// rows once, reusing the shared row between window rows); phase 2 transforms one tile per slot
// from LDS (channel-fastest, conflict-free) and writes V with 128-B coalesced stores.
constexpr int kPoolCg = 32, kPoolSlots = 10, kPoolThreads = kPoolCg * kPoolSlots, kPoolMaxWq = 40;
__global__ void __launch_bounds__(kPoolThreads) wino_in_pool_kernel(const float* __restrict__ c1,
                                                                    float* __restrict__ V, WinoPoolArgs g) {
  __shared__ float win[kN][kPoolMaxWq][kPoolCg];
  const int cgs = g.C / kPoolCg;
  const int cg = blockIdx.x % cgs;
  const int ti = (blockIdx.x / cgs) % g.ty;
  const int n = blockIdx.x / (cgs * g.ty);
  const int c = threadIdx.x % kPoolCg, slot = threadIdx.x / kPoolCg;
  const int ch = cg * kPoolCg + c;
  const float* img = c1 + static_cast<size_t>(n) * g.H1 * g.W1 * g.C + ch;
  // phase 1: window rows ti*3 .. ti*3+6, all Wq columns
  for (int xx = slot; xx < g.Wq; xx += kPoolSlots) {
    const int px = xx - g.pad;
    const bool col_ok = px >= 0 && px < g.Wp;
    float last = 0.f;
    bool have_last = false;
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int yy = ti * kM + u;
      const int pr = yy + g.q_lo;
      float v = 0.f;
      if (col_ok && yy < g.Hq && pr >= g.p1_lo && pr < g.p1_hi) {
        const int lr = 2 * pr - g.c1_lo;
        auto hmax = [&](int r) {
          const float* q = img + (static_cast<size_t>(r) * g.W1 + 2 * px) * g.C;
          return fmaxf(fmaxf(q[0], q[g.C]), q[2 * g.C]);
        };
        const float h0 = have_last ? last : hmax(lr);
        const float h1 = hmax(lr + 1), h2 = hmax(lr + 2);
        v = fmaxf(fmaxf(h0, h1), h2);
        last = h2;
        have_last = true;
      } else {
        have_last = false;
      }
      win[u][xx][c] = v;
    }
  }
  __syncthreads();
  // phase 2: one tile per slot
  for (int tj = slot; tj < g.tx; tj += kPoolSlots) {
    float t[kN][kN];
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int v = 0; v < kN; ++v) t[a][v] = 0.f;
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      float row[kN];
#pragma unroll
      for (int v = 0; v < kN; ++v) {
        const int xx = tj * kM + v;
        row[v] = xx < g.Wq ? win[u][xx][c] : 0.f;
      }
#pragma unroll
      for (int a = 0; a < kN; ++a)
        if (wino::kBT[a][u] != 0.f)
#pragma unroll
          for (int v = 0; v < kN; ++v) t[a][v] = fmaf(wino::kBT[a][u], row[v], t[a][v]);
    }
    const int p = (n * g.ty + ti) * g.tx + tj;
    float* out = V + static_cast<size_t>(p) * (kN * kN) * g.C + ch;
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int b = 0; b < kN; ++b) {
        float s2 = 0.f;
#pragma unroll
        for (int v = 0; v < kN; ++v)
          if (wino::kBT[b][v] != 0.f) s2 = fmaf(wino::kBT[b][v], t[a][v], s2);
        out[static_cast<size_t>(a * kN + b) * g.C] = s2;
      }
  }
}

__global__ void __launch_bounds__(kT) wino_out_kernel(const float* __restrict__ Mt, const float* __restrict__ bias,
                                                      float* __restrict__ y, int N, int Ho, int Wo, int K, int ty,
                                                      int tx, int relu) {
  const int K4 = K / 4;
  const long total = static_cast<long>(N) * ty * tx * K4;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int k4 = static_cast<int>(i % K4);
    const long p = i / K4;
    const int tj = static_cast<int>(p % tx);
    const long q = p / tx;
    const int ti = static_cast<int>(q % ty);
    const int n = static_cast<int>(q / ty);
    const float* src = Mt + static_cast<size_t>(p) * (kN * kN) * K + k4 * 4;
    // t = A^T M (3 x 7), then Y = t A (3 x 3)
    f32x4 t[kM][kN];
#pragma unroll
    for (int i3 = 0; i3 < kM; ++i3)
#pragma unroll
      for (int b = 0; b < kN; ++b) t[i3][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < kN; ++a)
#pragma unroll
      for (int b = 0; b < kN; ++b) {
        const f32x4 m = *reinterpret_cast<const f32x4*>(src + static_cast<size_t>(a * kN + b) * K);
#pragma unroll
        for (int i3 = 0; i3 < kM; ++i3)
          if (wino::kAT[i3][a] != 0.f) t[i3][b] += wino::kAT[i3][a] * m;
      }
    const f32x4 bv = bias ? *reinterpret_cast<const f32x4*>(bias + k4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i3 = 0; i3 < kM; ++i3) {
      const int oy = ti * kM + i3;
      if (oy >= Ho) break;
#pragma unroll
      for (int j3 = 0; j3 < kM; ++j3) {
        const int ox = tj * kM + j3;
        if (ox >= Wo) break;
        f32x4 s = bv;
#pragma unroll
        for (int b = 0; b < kN; ++b)
          if (wino::kAT[j3][b] != 0.f) s += wino::kAT[j3][b] * t[i3][b];
        if (relu) s = f32x4{fmaxf(s.x, 0.f), fmaxf(s.y, 0.f), fmaxf(s.z, 0.f), fmaxf(s.w, 0.f)};
        *reinterpret_cast<f32x4*>(y + ((static_cast<size_t>(n) * Ho + oy) * Wo + ox) * K + k4 * 4) = s;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused batched GEMM + output transform. A workgroup owns 64 tiles x 64 filters (2x2 waves of a
// 32x32 v_mfma_f32_32x32x2_f32 tile) and walks the 49 transform points ab: for each ab it forms
// M_ab = V_ab[64 x Cg] . U_ab[Cg x 64] in one 16-register accumulator (K = Cg in LDS-staged BK=32
// slices, same staging/k-permutation as conv_mfma.hip), then folds it straight into the 3x3
// outputs: Y[i][j] += A^T[i][a] A^T[j][b] M_ab. M never touches memory (it was 520 MB per 128
// images as a separate GEMM output), and bias + ReLU + the NHWC store happen once at the end.
// Per lane: 16 (tile, filter) pairs x 9 outputs = 144 Y registers + 16 accumulators.
constexpr int kFB = 64;  // tiles x filters per fused workgroup

struct FusedArgs {
  const float* V;      // [P][49][C]
  const float* U;      // packed [49*groups][kpad_n][kpad]
  const float* bias;   // [K]
  float* y;            // [N][Ho][Wo][K]
  int P, C, Cg, Kg, K, groups, kpad, kpad_n;
  int N, Ho, Wo, ty, tx, relu, n_ptiles, n_ntiles;
  int prio;  // bit0: s_setprio(1) around each slice's MFMAs (guide technique T5); bit8: interleaved fold.
             // Cost probes of the
             // LDS-DMA kernel (wrong results; never set in production): bit4 no fold, bit5 no DMA
             // refills, bit6 no per-slice barrier (only with bit5), bit7 no epilogue stores
  // Tail split (LDS-DMA kernel, non-IL): this launch covers point tiles [pt_base, pt_base +
  // n_ptiles); with nsplit > 1, blockIdx.y = s takes transform points [49 s / nsplit, 49 (s+1) /
  // nsplit) and stores its raw fold Y (no bias / ReLU) to slab s of `slab`, summed by
  // wino_split_reduce_kernel.
  int pt_base, nsplit;
  float* slab;
  int sk_groups;  // stream-K (wino_fused_sk_kernel): number of point ranges J
  int vbytes, ubytes;  // > 0: V / U sizes in bytes (< 2^31): operands by buffer_load ... lds; 0: global_load_lds
};

// A^T indexed by the runtime transform point: a copy of wino::kAT in constant memory (scalar loads).
struct ATTable {
  float v[kM][kN];
};
constexpr ATTable make_at() {
  ATTable t{};
  for (int i = 0; i < kM; ++i)
    for (int j = 0; j < kN; ++j) t.v[i][j] = wino::kAT[i][j];
  return t;
}
__constant__ ATTable c_at = make_at();
#define c_AT c_at.v

// Fold coefficients per transform point: coef[ab][i*kM + j] = A^T[i][a] * A^T[j][b] (float product,
// the value the runtime-indexed fold computes).
struct CoefTable {
  float v[kN * kN][kM * kM];
};
constexpr CoefTable make_coef() {
  CoefTable t{};
  for (int ab = 0; ab < kN * kN; ++ab)
    for (int i = 0; i < kM; ++i)
      for (int j = 0; j < kM; ++j) t.v[ab][i * kM + j] = wino::kAT[i][ab / kN] * wino::kAT[j][ab % kN];
  return t;
}
__constant__ CoefTable c_coef = make_coef();

template <int BK, bool XCD>
__global__ void __launch_bounds__(256) wino_fused_kernel(FusedArgs a) {
  using f32x16 = __attribute__((ext_vector_type(16))) float;
  constexpr int LDA = BK + 4;          // +16 B per row: conflict-free ds_read_b128 (row stride odd in 16 B)
  constexpr int U4 = BK / 4;           // float4 units per staged row
  constexpr int NJ = kFB * U4 / 256;   // float4 loads per thread per operand
  static_assert(NJ * 256 == kFB * U4, "BK must be a multiple of 16");
  __shared__ __attribute__((aligned(16))) float lds[2 * kFB * LDA];
  float* As = lds;
  float* Bs = lds + kFB * LDA;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = blockIdx.z;
  int pt, nt;
  if constexpr (XCD) {
    // the n_ntiles blocks that re-read one V slab run on one XCD (blocks b, b+8, ... share an L2)
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    nt = j % a.n_ntiles;
    pt = (j / a.n_ntiles) * 8 + xcd;
    if (pt >= a.n_ptiles) return;
  } else {
    pt = blockIdx.x / a.n_ntiles;
    nt = blockIdx.x - pt * a.n_ntiles;
  }
  const int p0 = pt * kFB, n0 = nt * kFB;
  int srow[NJ], scol[NJ], prow[NJ];
  unsigned pok = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int u = tid + 256 * j;
    srow[j] = u / U4;
    scol[j] = (u - srow[j] * U4) * 4;
    const int p = p0 + srow[j];
    pok |= (p < a.P ? 1u : 0u) << j;
    prow[j] = p < a.P ? p : 0;
  }
  const float* Vg = a.V + g * a.Cg;
  const int ksteps = a.kpad / BK;
  const int total = kN * kN * ksteps;
  f32x4 ra[NJ], rb[NJ];
  auto load = [&](int it) {
    const int ab = it / ksteps, kk = (it - ab * ksteps) * BK;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int kc = kk + scol[j];
      const bool kin = kc < a.Cg;  // K padding (Cg not a multiple of BK)
      ra[j] = *reinterpret_cast<const f32x4*>(Vg + (static_cast<size_t>(prow[j]) * (kN * kN) + ab) * a.C +
                                             (kin ? kc : 0));
      if (!kin || !((pok >> j) & 1u)) ra[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      rb[j] = *reinterpret_cast<const f32x4*>(
          a.U + (static_cast<size_t>(ab * a.groups + g) * a.kpad_n + n0 + srow[j]) * a.kpad + kc);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      *reinterpret_cast<f32x4*>(As + srow[j] * LDA + scol[j]) = ra[j];
      *reinterpret_cast<f32x4*>(Bs + srow[j] * LDA + scol[j]) = rb[j];
    }
  };
  const int r = lane & 31, h = lane >> 5;
  const float* a_rd = As + (wm * 32 + r) * LDA + h * (BK / 2);
  const float* b_rd = Bs + (wn * 32 + r) * LDA + h * (BK / 2);
  f32x16 acc = {};
  float Y[9][16];
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int e = 0; e < 16; ++e) Y[q][e] = 0.f;

  load(0);
  store();
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    if (it + 1 < total) load(it + 1);
#pragma unroll
    for (int s4 = 0; s4 < BK / 8; ++s4) {
      const f32x4 af = *reinterpret_cast<const f32x4*>(a_rd + s4 * 4);
      const f32x4 bf = *reinterpret_cast<const f32x4*>(b_rd + s4 * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
    const int ab = it / ksteps;
    if (it - ab * ksteps == ksteps - 1) {
      // fold M_ab into the 3x3 outputs (coefficients are wave-uniform: scalar registers)
      const int aa = ab / kN, bb = ab - aa * kN;
      float co[9];
#pragma unroll
      for (int i3 = 0; i3 < kM; ++i3)
#pragma unroll
        for (int j3 = 0; j3 < kM; ++j3) co[i3 * kM + j3] = c_AT[i3][aa] * c_AT[j3][bb];
#pragma unroll
      for (int q = 0; q < 9; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) Y[q][e] = fmaf(co[q], acc[e], Y[q][e]);
      acc = f32x16{};
    }
    __syncthreads();
    if (it + 1 < total) {
      store();
      __syncthreads();
    }
  }
  // epilogue: lane holds filter f (col) and tiles (rows) (e&3) + 8*(e>>2) + 4h
  const int f = n0 + wn * 32 + r;
  if (f >= a.Kg) return;
  const int fk = g * a.Kg + f;
  const float bv = a.bias ? a.bias[fk] : 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int p = p0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (p >= a.P) continue;
    const int tj = p % a.tx;
    const int q = p / a.tx;
    const int ti = q % a.ty;
    const int n = q / a.ty;
#pragma unroll
    for (int i3 = 0; i3 < kM; ++i3) {
      const int oy = ti * kM + i3;
      if (oy >= a.Ho) break;
#pragma unroll
      for (int j3 = 0; j3 < kM; ++j3) {
        const int ox = tj * kM + j3;
        if (ox >= a.Wo) break;
        float v = Y[i3 * kM + j3][e] + bv;
        if (a.relu) v = fmaxf(v, 0.f);
        a.y[((static_cast<size_t>(n) * a.Ho + oy) * a.Wo + ox) * a.K + fk] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Same computation, staged by LDS-DMA. The register-staged kernel above needs ~246 VGPR+AGPR
// (144 Y + 16 acc + 24 staging + addressing), so it runs at 2 waves/SIMD and every K slice's
// global loads must land within one slice of MFMAs. Here the operand tiles go global -> LDS with
// global_load_lds_dwordx4 (no staging registers) into a 3-deep ring: slice it+2 is in flight
// while slice it computes, retired by a counted `s_waitcnt vmcnt` and ONE raw s_barrier per slice
// (a __syncthreads() would drain the in-flight DMA: cdna_hip_programming.md §5 "Pipelining
// across barriers"). The freed registers hold a second accumulator, so the 144-FMA output fold
// of point ab runs on the VALU while the MFMAs of point ab+1 are in flight.
//
// LDS image: rows of BK floats, unpadded (the DMA writes lane-linear 1 KiB pieces); the 16-byte
// unit u of row r is stored at unit u ^ ((r >> 2) & 3), which makes the ds_read_b128 lane groups
// of the 32x32 fragment reads hit 16 distinct bank quads. The swizzle is applied on the global
// source address of each lane.
using lds_f32 = __attribute__((address_space(3))) float;
using lds_void = __attribute__((address_space(3))) void;
// 16 B per lane, global -> LDS (lane i lands at lds + 16*i; lds must be wave-uniform)
__device__ __forceinline__ void glds16(const float* g, lds_f32* lds) { __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0); }
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// One fold step on a register pair: y += c * (a0, a1). SF = two scalar v_fma_f32 (this file builds
// with -fno-slp-vectorize, so they stay scalar), else one v_pk_fma_f32. Bit-identical either way.
template <bool SF>
__device__ __forceinline__ void fma2(f32x2& y, float c, float a0, float a1) {
  if constexpr (SF) {
    y.x = fmaf(c, a0, y.x);
    y.y = fmaf(c, a1, y.y);
  } else {
    y = __builtin_elementwise_fma(f32x2{c, c}, f32x2{a0, a1}, y);
  }
}

// One unit of the LDS-DMA kernel: point tile pt (64 tiles), filter tile nt (64 filters), conv group
// g, over transform points [pb, pe). slab == nullptr: the unit covers all 49 points and ends in the
// bias + ReLU + NHWC epilogue; otherwise the raw fold Y of the range goes to `slab` as [q][tile]
// [filter] (9 x 64 x 64 floats) for a reduce kernel. IL: full units run the interleaved-fold schedule.
// IL_MODE: 0 = generic point-range schedule only, 1 = interleaved-fold schedule only (whole units),
// 2 = interleaved for whole units, generic for partial ranges (chosen at run time).
template <int BK, int IL_MODE, bool SF>
__device__ __forceinline__ void fused_glds_unit(const FusedArgs& a, float* lds, int pt, int nt, int g, int pb, int pe,
                                                float* slab) {
  using f32x16 = __attribute__((ext_vector_type(16))) float;
  constexpr int U4 = BK / 4;              // 16-B units per row
  constexpr int NI = kFB * U4 / 256;      // DMA instructions per thread per operand
  static_assert(NI * 256 == kFB * U4 && U4 % 4 == 0, "BK must be a multiple of 16");
  constexpr int TILE = kFB * BK;          // floats per operand tile
  constexpr int STAGE = 2 * TILE;         // A tile | B tile
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int wm = wave >> 1, wn = wave & 1;
  const int p0 = pt * kFB, n0 = nt * kFB;

  // per-lane source offsets of this thread's NI A units and NI B units (swizzled unit order)
  int aoff[NI], boff[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int U = (j * 4 + wave) * 64 + lane;
    const int row = U / U4;
    const int u = (U - row * U4) ^ ((row >> 2) & 3);
    const int p = p0 + row;
    aoff[j] = (p < a.P ? p : 0) * (kN * kN) * a.C + 4 * u;
    boff[j] = (n0 + row) * a.kpad + 4 * u;
  }
  const float* Vg = a.V + g * a.Cg;
  // the interleaved schedule only runs at kpad == 2 * BK (launch condition): a compile-time slice count
  const int ksteps = IL_MODE == 1 ? 2 : a.kpad / BK;
  const int it0 = pb * ksteps, total = pe * ksteps;  // K slices [it0, total) (all 49 points unless split)
  lds_f32* lds3 = (lds_f32*)(lds);  // generic -> LDS address space (C-style cast required)

  // buffer_load ... lds when V and U fit 32-bit byte offsets (a.vbytes > 0): the per-lane offsets
  // stay in VGPRs once, the per-slice offset is scalar (no 64-bit VALU address per DMA)
#if __HIP_DEVICE_COMPILE__  // the buffer-resource type exists in the device pass only
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.V), 0, a.vbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
#endif
  auto issue = [&](int it) {
    const int ab = it / ksteps, kk = (it - ab * ksteps) * BK;
    lds_f32* st = lds3 + (it % 3) * STAGE;
#if __HIP_DEVICE_COMPILE__
    if (a.vbytes > 0) {
      const int vso = (g * a.Cg + ab * a.C + kk) * 4;
      const int uso = ((ab * a.groups + g) * a.kpad_n * a.kpad + kk) * 4;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (lds_void*)(st + (j * 4 + wave) * 256), 16, aoff[j] * 4, vso, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)(st + TILE + (j * 4 + wave) * 256), 16, boff[j] * 4,
                                                 uso, 0, 0);
      }
      return;
    }
#endif
    const float* va = Vg + ab * a.C + kk;
    const float* ub = a.U + static_cast<size_t>(ab * a.groups + g) * a.kpad_n * a.kpad + kk;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      glds16(va + aoff[j], st + (j * 4 + wave) * 256);
      glds16(ub + boff[j], st + TILE + (j * 4 + wave) * 256);
    }
  };

  const int r = lane & 31, h = lane >> 5;
  const int swz = (r >> 2) & 3;  // rows wm*32 + r and wn*32 + r share it
  int rd[BK / 8];                // unit (h*BK/8 + s4) of my row, swizzled, in floats
#pragma unroll
  for (int s4 = 0; s4 < BK / 8; ++s4) rd[s4] = 4 * ((h * (BK / 8) + s4) ^ swz);
  const int a_row = (wm * 32 + r) * BK, b_row = TILE + (wn * 32 + r) * BK;

  // Y[q][e2]: output q of accumulator rows 2*e2 and 2*e2+1 (pairs: one v_pk_fma_f32 per 2 rows,
  // or two v_fma_f32 with SF)
  f32x2 Y[9][8];
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) Y[q][e2] = f32x2{0.f, 0.f};
  f32x16 acc0 = {}, acc1 = {};

  auto mfma_slice = [&](int it, f32x16& acc) {
    const float* base = lds + (it % 3) * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < BK / 8; ++s4) {
      const f32x4 af = *reinterpret_cast<const f32x4*>(base + a_row + rd[s4]);
      const f32x4 bf = *reinterpret_cast<const f32x4*>(base + b_row + rd[s4]);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
  };
  // coefficients are wave-uniform (scalar registers): a zero one (152 of the 441 coefficient x
  // point pairs) skips its 16 FMAs with a scalar branch
  auto fold = [&](int ab, f32x16& acc) {
    if (a.prio & 16) {  // probe: keep the accumulator live, skip the output-transform FMAs
      Y[0][0] += f32x2{acc[0], acc[1]};
      acc = f32x16{};
      return;
    }
    const int aa = ab / kN, bb = ab - aa * kN;
#pragma unroll
    for (int i3 = 0; i3 < kM; ++i3)
#pragma unroll
      for (int j3 = 0; j3 < kM; ++j3) {
        const float c = c_AT[i3][aa] * c_AT[j3][bb];
        if (c != 0.f) {
#pragma unroll
          for (int e2 = 0; e2 < 8; ++e2) fma2<SF>(Y[i3 * kM + j3][e2], c, acc[2 * e2], acc[2 * e2 + 1]);
        }
      }
    acc = f32x16{};
  };
  // one K slice: retire slice it (counted wait + barrier), refill the ring slot freed by it-1
  auto step = [&](int it, f32x16& acc) {
    if (it + 1 < total)
      wait_vmcnt<2 * NI>();
    else
      wait_vmcnt<0>();
    if ((a.prio & 96) != 96) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // keep the DMA refill and the ds_reads below the barrier
    if (it + 2 < total && !(a.prio & 32)) issue(it + 2);
    if (a.prio & 1) __builtin_amdgcn_s_setprio(1);
    mfma_slice(it, acc);
    if (a.prio & 1) __builtin_amdgcn_s_setprio(0);
  };

  // IL: the fold of point fab rides inside the first slice of the next point, branch-free (zero
  // coefficients included: +0 leaves Y bit-identical), 3 packed FMAs after each MFMA, so the VALU
  // work issues while the wave's MFMAs occupy the matrix pipe instead of after them.
  // mfma_slice with the fragments of group s4+1 read while group s4's MFMAs run
  auto mfma_slice_pf = [&](int it, f32x16& acc) {
    const float* base = lds + (it % 3) * STAGE;
    f32x4 af[2], bf[2];
    af[0] = *reinterpret_cast<const f32x4*>(base + a_row + rd[0]);
    bf[0] = *reinterpret_cast<const f32x4*>(base + b_row + rd[0]);
#pragma unroll
    for (int s4 = 0; s4 < BK / 8; ++s4) {
      if (s4 + 1 < BK / 8) {
        af[(s4 + 1) & 1] = *reinterpret_cast<const f32x4*>(base + a_row + rd[s4 + 1]);
        bf[(s4 + 1) & 1] = *reinterpret_cast<const f32x4*>(base + b_row + rd[s4 + 1]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s4 & 1][s], bf[s4 & 1][s], acc, 0, 0, 0);
    }
  };
  // IL (ksteps == 2 only): the fold of point fab rides inside the first slice of the next point,
  // branch-free (zero coefficients included: +0 leaves Y bit-identical), 3 packed FMAs after each
  // MFMA, so the VALU work issues while the wave's MFMAs occupy the matrix pipe instead of after
  // them. Straight-line loop body: in-loop slices always wait vmcnt(2*NI) and always refill.
  auto slice_fold = [&](int it, f32x16& acc, int fab, f32x16& facc) {
    float cq[kM * kM];
#pragma unroll
    for (int q = 0; q < kM * kM; ++q) cq[q] = c_coef.v[fab][q];
    const float* base = lds + (it % 3) * STAGE;
    static_assert(IL_MODE == 0 || (BK / 8) * 4 * 3 >= kM * kM * 8, "fold FMAs must fit behind the slice's MFMAs");
    // fragments of group s4+1 are read while group s4's MFMAs run (two register sets)
    f32x4 af[2], bf[2];
    af[0] = *reinterpret_cast<const f32x4*>(base + a_row + rd[0]);
    bf[0] = *reinterpret_cast<const f32x4*>(base + b_row + rd[0]);
#pragma unroll
    for (int s4 = 0; s4 < BK / 8; ++s4) {
      if (s4 + 1 < BK / 8) {
        af[(s4 + 1) & 1] = *reinterpret_cast<const f32x4*>(base + a_row + rd[s4 + 1]);
        bf[(s4 + 1) & 1] = *reinterpret_cast<const f32x4*>(base + b_row + rd[s4 + 1]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s4 & 1][s], bf[s4 & 1][s], acc, 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int j = (s4 * 4 + s) * 3 + t;
          if (j < kM * kM * 8) {
            const int q = j >> 3, e2 = j & 7;
            fma2<SF>(Y[q][e2], cq[q], facc[2 * e2], facc[2 * e2 + 1]);
          }
        }
      }
    }
    facc = f32x16{};
  };
  auto step_mid = [&](int it, f32x16& acc, int fab, f32x16* facc) {  // it + 2 < total
    wait_vmcnt<2 * NI>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(it + 2);
    if (a.prio & 1) __builtin_amdgcn_s_setprio(1);
    if (facc)
      slice_fold(it, acc, fab, *facc);
    else
      mfma_slice_pf(it, acc);
    if (a.prio & 1) __builtin_amdgcn_s_setprio(0);
  };

  issue(it0);
  if (it0 + 1 < total) issue(it0 + 1);
  bool il_sched;
  if constexpr (IL_MODE == 1)
    il_sched = true;  // the caller only passes whole units
  else if constexpr (IL_MODE == 2)
    il_sched = pb == 0 && pe == kN * kN;
  else
    il_sched = false;
  if (IL_MODE != 0 && il_sched) {
    // acc1 is zero before point 1: the first fold adds +0 (ab = 0's coefficients) and changes nothing
    for (int ab = 0; ab + 1 < kN * kN; ab += 2) {
      const int it = 2 * ab;
      step_mid(it, acc0, ab > 0 ? ab - 1 : 0, &acc1);
      step_mid(it + 1, acc0, 0, nullptr);
      step_mid(it + 2, acc1, ab, &acc0);
      step_mid(it + 3, acc1, 0, nullptr);
    }
    // point 48: slices 96 (fold of 47 inside) and 97 (last: no refill, full drain)
    wait_vmcnt<2 * NI>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    slice_fold(total - 2, acc0, kN * kN - 2, acc1);
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    mfma_slice_pf(total - 1, acc0);
  } else {
    // ab pairs: the last point pe-1 and every second one before it accumulate in acc0, the others
    // in acc1 (an even count starts with a lone point in acc1, so acc1 is dead after the loop); the
    // fold of the previous point is issued after the first slice of the next one, so the VALU work
    // overlaps in-flight MFMAs. All 49 points: the original order (pb = 0 in acc0).
    int it = it0, ab0 = pb;
    if (((pe - pb) & 1) == 0) {
      for (int ks = 0; ks < ksteps; ++ks, ++it) step(it, acc1);
      ab0 = pb + 1;
    }
    for (int ab = ab0; ab < pe; ab += 2) {
      for (int ks = 0; ks < ksteps; ++ks, ++it) {
        step(it, acc0);
        if (ks == 0 && ab > pb) fold(ab - 1, acc1);
      }
      if (ab + 1 < pe) {
        for (int ks = 0; ks < ksteps; ++ks, ++it) {
          step(it, acc1);
          if (ks == 0) fold(ab, acc0);
        }
      }
    }
  }
  // the last point is still unfolded, in acc0
  fold(pe - 1, acc0);

  if (slab) {  // partial point range: raw Y, [q][tile][filter]
    float* sl = slab;
#pragma unroll
    for (int q = 0; q < kM * kM; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        sl[(q * kFB + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * kFB + wn * 32 + r] = Y[q][e >> 1][e & 1];
    return;
  }

  // Epilogue: bias + ReLU, then one LDS transpose per output position q so each lane stores whole
  // 16-B filter groups (4 dwordx4 per lane per q instead of 16 single-dword stores, which were
  // store-issue-bound). D layout: lane (r, h) holds filter n0 + wn*32 + r of wave tiles
  // wm*32 + (e&3) + 8*(e>>2) + 4h. Kg % 4 == 0 (wino_eligible), so a 4-filter group is all in or
  // all past Kg.
  __syncthreads();  // the ring is idle (last slice waited with vmcnt(0)); reuse it as scratch
  constexpr int kTS = 32 + 4;
  float* tr = lds + wave * 32 * kTS;
  const int fb = n0 + wn * 32;  // first filter of this wave (within the group)
  const float bv = (a.bias && fb + r < a.Kg) ? a.bias[g * a.Kg + fb + r] : 0.f;
  int oy0[4], ox0[4], img[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + wm * 32 + ((k * 64 + lane) >> 3);
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = (p < a.P && !(a.prio & 128)) ? (pq % a.ty) * kM : (1 << 28);  // out of range: never stored
    ox0[k] = tj * kM;
    img[k] = pq / a.ty;
  }
  const int grp = 4 * (lane & 7);
  const bool fin = fb + grp < a.Kg;
#pragma unroll
  for (int q = 0; q < kM * kM; ++q) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float v = Y[q][e >> 1][e & 1] + bv;
      if (a.relu) v = fmaxf(v, 0.f);
      tr[((e & 3) + 8 * (e >> 2) + 4 * h) * kTS + r] = v;
    }
    // same-wave LDS accesses complete in order (reads see the writes; later writes cannot overtake)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) >> 3) * kTS + grp);
      const int oy = oy0[k] + q / kM, ox = ox0[k] + q % kM;
      if (fin && oy < a.Ho && ox < a.Wo)
        *reinterpret_cast<f32x4*>(a.y + ((static_cast<size_t>(img[k]) * a.Ho + oy) * a.Wo + ox) * a.K + g * a.Kg + fb +
                                  grp) = v4;
    }
  }
}

template <int BK, bool XCD, bool IL, bool SF>
__global__ void __launch_bounds__(256, 2) wino_fused_glds_kernel(FusedArgs a) {  // 2 waves/SIMD
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int g = blockIdx.z;
  int pt, nt;
  if constexpr (XCD) {
    // the n_ntiles workgroups that read one V slab get equal blockIdx.x % 8 (one XCD, one L2)
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    nt = j % a.n_ntiles;
    pt = (j / a.n_ntiles) * 8 + xcd;
    if (pt >= a.n_ptiles) return;  // whole workgroup, before any DMA or barrier
  } else {
    pt = blockIdx.x / a.n_ntiles;
    nt = blockIdx.x - pt * a.n_ntiles;
  }
  const int ptl = pt;  // point tile within this launch (slab index)
  // transform points of this workgroup: all 49, or slice blockIdx.y of a tail split
  const int nsplit = a.nsplit > 1 ? a.nsplit : 1, sidx = nsplit > 1 ? blockIdx.y : 0;
  const int pb = kN * kN * sidx / nsplit, pe = kN * kN * (sidx + 1) / nsplit;
  float* sl = a.slab ? a.slab + ((((static_cast<size_t>(g) * nsplit + sidx) * a.n_ptiles + ptl) * a.n_ntiles + nt) *
                                 kM * kM) * (kFB * kFB)
                     : nullptr;
  fused_glds_unit<BK, IL ? 1 : 0, SF>(a, lds, pt + a.pt_base, nt, g, pb, pe, sl);
}

// Stream-K schedule of the same units (Knobs::wino_sk; conv groups == 1). The 49 * n_ptiles
// (point tile, transform point) pairs are cut into J equal contiguous ranges, one per group of
// n_ntiles workgroups (one per filter tile, all on one XCD, so a V slab is read by one L2), with J
// a whole number of workgroups per CU: every CU gets the same MFMA work, whatever the batch (the
// data-parallel grid leaves CUs with one workgroup next to CUs with two: 324 workgroups on 256 CUs
// at 64 images). A range covers whole point tiles (the fused epilogue) and at most two partial ones
// (its first and last), whose raw Y go to the group's two slab slots; wino_sk_reduce_kernel sums
// the slots of every split point tile in group order (deterministic) and stores act(sum + bias).
__device__ __forceinline__ long sk_start(long j, long T, int J) { return j * T / J; }

template <bool SF, bool IL>
__global__ void __launch_bounds__(256, 2) wino_fused_sk_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles;
  const int j = (jb / a.n_ntiles) * 8 + xcd;  // range index
  if (j >= a.sk_groups) return;               // whole workgroup, before any DMA or barrier
  const long T = static_cast<long>(a.n_ptiles) * (kN * kN);
  const long end = sk_start(j + 1, T, a.sk_groups);
  float* slots = a.slab + static_cast<size_t>(j * a.n_ntiles + nt) * 2 * (kM * kM * kFB * kFB);
  bool first = true;
  for (long x = sk_start(j, T, a.sk_groups); x < end;) {
    const int pt = static_cast<int>(x / (kN * kN)), pb = static_cast<int>(x - static_cast<long>(pt) * (kN * kN));
    const int pe = static_cast<int>(min(static_cast<long>(kN * kN), end - static_cast<long>(pt) * (kN * kN)));
    float* sl = (pb == 0 && pe == kN * kN) ? nullptr : slots + (first ? 0 : kM * kM * kFB * kFB);
    if (!first) __syncthreads();  // the previous unit's epilogue / last slices are done with the LDS
    fused_glds_unit<48, IL ? 2 : 0, SF>(a, lds, pt, nt, 0, pb, pe, sl);
    first = false;
    x = static_cast<long>(pt) * (kN * kN) + pe;
  }
}

// ---------------------------------------------------------------------------------------------
// The same fused GEMM on v_mfma_f32_16x16x4_f32 with 8 waves: the 64-tile x 64-filter workgroup is
// 4 (tiles) x 2 (filters) waves of 16 tiles x 32 filters (two 16x16 blocks). The fold registers
// halve (9 x 8 per lane), so two 512-thread workgroups (16 waves, 4 per SIMD) fit a CU at the same
// bytes per MAC as the 4-wave kernel above. Per K slice (48 channels) the 12 A and 12 B DMA
// instructions are dealt 3 per wave. 16x16x4 operands: lane l holds A[tile l&15][k], B[k][filter
// l&15] for its lane group g = l>>4, which at step t supplies k = 12g + t; D: filter l&15, tile
// 4g + reg. LDS rows rotate their 16-B units by 3*((r>>1)&3) mod 12: conflict-free for these reads
// (the rotation is applied to the DMA source address, as in conv1_wino.hip).
__device__ __forceinline__ int rot16(int row) { return 3 * ((row >> 1) & 3); }

template <int WMW, int WNW, bool XCD>
__global__ void __launch_bounds__(64 * WMW * WNW, 4) wino_fused_glds16_kernel(FusedArgs a) {  // 4 waves/SIMD
  constexpr int NW = WMW * WNW;               // waves per workgroup
  constexpr int BMT = 16 * WMW, BNT = 32 * WNW;  // tiles x filters per workgroup
  constexpr int BK = 48, U4 = BK / 4;
  constexpr int A_INS = BMT * U4 / 64, B_INS = BNT * U4 / 64, INS = A_INS + B_INS;
  constexpr int PW = (INS + NW - 1) / NW;     // DMA slots per wave (the last may be empty)
  constexpr int NS_HI = PW, NS_LO = INS % NW ? PW - 1 : PW;  // DMAs per slice: waves < INS % NW / the rest
  constexpr int A_FL = BMT * BK, B_FL = BNT * BK;
  constexpr int STAGE = A_FL + B_FL;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int wm = wave % WMW, wn = wave / WMW;
  const int g = blockIdx.z;
  int pt, nt;
  if constexpr (XCD) {
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    nt = j % a.n_ntiles;
    pt = (j / a.n_ntiles) * 8 + xcd;
    if (pt >= a.n_ptiles) return;  // whole workgroup, before any DMA or barrier
  } else {
    pt = blockIdx.x / a.n_ntiles;
    nt = blockIdx.x - pt * a.n_ntiles;
  }
  const int p0 = pt * BMT, n0 = nt * BNT;
  // DMA instruction q = wave + NW*i of the slice's INS (A_INS for A, then B_INS for B)
  int off[PW], dst[PW];
  bool isa[PW], has[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int q = wave + NW * i;
    has[i] = q < INS;
    isa[i] = q < A_INS;
    const int qq = has[i] ? (isa[i] ? q : q - A_INS) : 0;
    const int U = qq * 64 + lane;
    const int row = U / U4, su = U - row * U4;
    const int u = (su + U4 - rot16(row)) % U4;  // logical unit stored at slot su
    if (isa[i]) {
      const int p = p0 + row;
      off[i] = (p < a.P ? p : 0) * (kN * kN) * a.C + 4 * u;
    } else {
      off[i] = (n0 + row) * a.kpad + 4 * u;
    }
    dst[i] = (isa[i] ? 0 : A_FL) + qq * 256;
  }
  const bool hi = wave < INS % NW || INS % NW == 0;
  const float* Vg = a.V + g * a.Cg;
  const int ksteps = a.kpad / BK;
  const int total = kN * kN * ksteps;
  lds_f32* lds3 = (lds_f32*)(lds);
  auto issue = [&](int it) {
    const int ab = it / ksteps, kk = (it - ab * ksteps) * BK;
    const float* va = Vg + ab * a.C + kk;
    const float* ub = a.U + static_cast<size_t>(ab * a.groups + g) * a.kpad_n * a.kpad + kk;
    lds_f32* st = lds3 + (it % 3) * STAGE;
#pragma unroll
    for (int i = 0; i < PW; ++i)
      if (has[i]) glds16((isa[i] ? va : ub) + off[i], st + dst[i]);
  };

  const int r16 = lane & 15, lg = lane >> 4;
  const int a_row = (wm * 16 + r16) * BK, b_row0 = A_FL + (wn * 32 + r16) * BK, b_row1 = b_row0 + 16 * BK;
  int rd[3];
#pragma unroll
  for (int s4 = 0; s4 < 3; ++s4) rd[s4] = 4 * ((3 * lg + s4 + rot16(r16)) % U4);

  f32x2 Y[9][2][2];  // [q][block][register pair]
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int c = 0; c < 2; ++c) Y[q][c][0] = Y[q][c][1] = f32x2{0.f, 0.f};
  f32x4 acc0[2] = {}, acc1[2] = {};

  auto mfma_slice = [&](int it, f32x4 (&acc)[2]) {
    const float* base = lds + (it % 3) * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < 3; ++s4) {
      const f32x4 af = *reinterpret_cast<const f32x4*>(base + a_row + rd[s4]);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(base + b_row0 + rd[s4]);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(base + b_row1 + rd[s4]);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], b0[s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], b1[s], acc[1], 0, 0, 0);
      }
    }
  };
  auto fold = [&](int ab, f32x4 (&acc)[2]) {
    const int aa = ab / kN, bb = ab - aa * kN;
#pragma unroll
    for (int i3 = 0; i3 < kM; ++i3)
#pragma unroll
      for (int j3 = 0; j3 < kM; ++j3) {
        const float c = c_AT[i3][aa] * c_AT[j3][bb];
        if (c != 0.f) {
          const f32x2 c2 = {c, c};
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            Y[i3 * kM + j3][cb][0] = __builtin_elementwise_fma(c2, f32x2{acc[cb][0], acc[cb][1]}, Y[i3 * kM + j3][cb][0]);
            Y[i3 * kM + j3][cb][1] = __builtin_elementwise_fma(c2, f32x2{acc[cb][2], acc[cb][3]}, Y[i3 * kM + j3][cb][1]);
          }
        }
      }
    acc[0] = acc[1] = f32x4{};
  };
  auto step = [&](int it, f32x4 (&acc)[2]) {
    if (it + 1 >= total)
      wait_vmcnt<0>();
    else if (hi)
      wait_vmcnt<NS_HI>();  // slice it+1's DMAs of this wave stay in flight
    else
      wait_vmcnt<NS_LO>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 2 < total) issue(it + 2);
    if (a.prio & 1) __builtin_amdgcn_s_setprio(1);
    mfma_slice(it, acc);
    if (a.prio & 1) __builtin_amdgcn_s_setprio(0);
  };

  issue(0);
  if (total > 1) issue(1);
  int it = 0;
  for (int ab = 0; ab < kN * kN; ab += 2) {
    for (int ks = 0; ks < ksteps; ++ks, ++it) {
      step(it, acc0);
      if (ks == 0 && ab > 0) fold(ab - 1, acc1);
    }
    if (ab + 1 < kN * kN) {
      for (int ks = 0; ks < ksteps; ++ks, ++it) {
        step(it, acc1);
        if (ks == 0) fold(ab, acc0);
      }
    }
  }
  fold(kN * kN - 1, acc0);

  // epilogue: per output position q, transpose the wave's 16 tiles x 32 filters through LDS and
  // store 16-B filter groups (2 per lane)
  __syncthreads();
  constexpr int kTS = 32 + 4;
  float* tr = lds + wave * 16 * kTS;
  const int fb = n0 + wn * 32;
  float bv[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) bv[cb] = (a.bias && fb + cb * 16 + r16 < a.Kg) ? a.bias[g * a.Kg + fb + cb * 16 + r16] : 0.f;
  int oy0[2], ox0[2], img[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = p0 + wm * 16 + ((k * 64 + lane) >> 3);
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = p < a.P ? (pq % a.ty) * kM : (1 << 28);  // out of range: never stored
    ox0[k] = tj * kM;
    img[k] = pq / a.ty;
  }
  const int grp = 4 * (lane & 7);
  const bool fin = fb + grp < a.Kg;
#pragma unroll
  for (int q = 0; q < kM * kM; ++q) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        float v = Y[q][cb][reg >> 1][reg & 1] + bv[cb];
        if (a.relu) v = fmaxf(v, 0.f);
        tr[(4 * lg + reg) * kTS + cb * 16 + r16] = v;
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) >> 3) * kTS + grp);
      const int oy = oy0[k] + q / kM, ox = ox0[k] + q % kM;
      if (fin && oy < a.Ho && ox < a.Wo)
        *reinterpret_cast<f32x4*>(a.y + ((static_cast<size_t>(img[k]) * a.Ho + oy) * a.Wo + ox) * a.K + g * a.Kg + fb +
                                  grp) = v4;
    }
  }
}

template <int WMW, int WNW, bool XCD>
hipError_t launch_glds16(FusedArgs a, hipStream_t s) {
  constexpr int BMT = 16 * WMW, BNT = 32 * WNW;
  constexpr int kLds = 3 * (BMT + BNT) * 48 * sizeof(float);  // 3-slot ring of A|B tiles
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(wino_fused_glds16_kernel<WMW, WNW, XCD>), hipFuncAttributeMaxDynamicSharedMemorySize,
      kLds);
  if (attr != hipSuccess) return attr;
  a.n_ptiles = (a.P + BMT - 1) / BMT;
  a.n_ntiles = (a.Kg + BNT - 1) / BNT;
  if (a.n_ntiles * BNT > a.kpad_n) return hipErrorInvalidValue;  // B rows past the packed weights
  const dim3 grid((XCD ? (a.n_ptiles + 7) / 8 * 8 : a.n_ptiles) * a.n_ntiles, 1, a.groups);
  wino_fused_glds16_kernel<WMW, WNW, XCD><<<grid, 64 * WMW * WNW, kLds, s>>>(a);
  return hipGetLastError();
}

template <int BK, bool XCD, bool IL = false, bool SF = false>
hipError_t launch_glds(const FusedArgs& a, dim3 grid, hipStream_t s, int occ) {
  const size_t lds = occupancy_lds(3 * 2 * kFB * BK * sizeof(float), occ);  // 3-slot ring of A|B tiles
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(wino_fused_glds_kernel<BK, XCD, IL, SF>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  wino_fused_glds_kernel<BK, XCD, IL, SF><<<grid, 256, lds, s>>>(a);
  return hipGetLastError();
}

// Tail-split fixup: y = act(sum_s slab[s] + bias) for the split point tiles, slabs summed in slice
// order (deterministic); 4 filters per thread (16-B loads / store), the fused epilogue's NHWC store.
struct SplitReduceArgs {
  const float* slab;
  const float* bias;
  float* y;
  int nsplit, n_ptiles, n_ntiles, pt_base, groups;
  int P, Kg, K, Ho, Wo, ty, tx, relu;
};
__global__ void __launch_bounds__(256) wino_split_reduce_kernel(SplitReduceArgs r) {
  constexpr int F4 = kFB / 4;
  const long total = static_cast<long>(r.groups) * r.n_ptiles * r.n_ntiles * kM * kM * kFB * F4;
  const size_t sstride = static_cast<size_t>(r.n_ptiles) * r.n_ntiles * kM * kM * kFB * kFB;  // between slices
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += static_cast<long>(gridDim.x) * 256) {
    long t = i;
    const int f4 = static_cast<int>(t % F4);
    t /= F4;
    const int tl = static_cast<int>(t % kFB);
    t /= kFB;
    const int q = static_cast<int>(t % (kM * kM));
    t /= kM * kM;
    const int nt = static_cast<int>(t % r.n_ntiles);
    t /= r.n_ntiles;
    const int ptl = static_cast<int>(t % r.n_ptiles);
    const int g = static_cast<int>(t / r.n_ptiles);
    const int f = nt * kFB + f4 * 4;
    const int p = (r.pt_base + ptl) * kFB + tl;
    if (f >= r.Kg || p >= r.P) continue;
    const int tj = p % r.tx, pq = p / r.tx, ti = pq % r.ty, n = pq / r.ty;
    const int oy = ti * kM + q / kM, ox = tj * kM + q % kM;
    if (oy >= r.Ho || ox >= r.Wo) continue;
    const float* src = r.slab + (((static_cast<size_t>(g) * r.nsplit * r.n_ptiles + ptl) * r.n_ntiles + nt) * kM * kM + q) *
                                    (kFB * kFB) + tl * kFB + f4 * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < r.nsplit; ++sl) v += *reinterpret_cast<const f32x4*>(src + sl * sstride);
    if (r.bias) v += *reinterpret_cast<const f32x4*>(r.bias + g * r.Kg + f);
    if (r.relu) v = f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
    *reinterpret_cast<f32x4*>(r.y + ((static_cast<size_t>(n) * r.Ho + oy) * r.Wo + ox) * r.K + g * r.Kg + f) = v;
  }
}

// Stream-K fixup: y = act(sum over the ranges j covering point tile pt of their slab slot + bias)
// for every split point tile (covered by more than one range); ranges in order (deterministic).
struct SkReduceArgs {
  const float* slab;
  const float* bias;
  float* y;
  int J, n_ptiles, n_ntiles;
  int P, Kg, K, Ho, Wo, ty, tx, relu;
};
__device__ __forceinline__ int sk_range_of(long x, long T, int J) {  // j with start(j) <= x < start(j+1)
  int j = static_cast<int>(x * J / T);
  if (j + 1 < J && sk_start(j + 1, T, J) <= x) ++j;
  return j;
}
__global__ void __launch_bounds__(256) wino_sk_reduce_kernel(SkReduceArgs r) {
  constexpr int F4 = kFB / 4, Q = kM * kM;
  const long T = static_cast<long>(r.n_ptiles) * (kN * kN);
  const long total = static_cast<long>(r.n_ptiles) * r.n_ntiles * Q * kFB * F4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += static_cast<long>(gridDim.x) * 256) {
    long t = i;
    const int f4 = static_cast<int>(t % F4);
    t /= F4;
    const int tl = static_cast<int>(t % kFB);
    t /= kFB;
    const int q = static_cast<int>(t % Q);
    t /= Q;
    const int nt = static_cast<int>(t % r.n_ntiles);
    const int pt = static_cast<int>(t / r.n_ntiles);
    const long x0 = static_cast<long>(pt) * (kN * kN);
    const int jlo = sk_range_of(x0, T, r.J), jhi = sk_range_of(x0 + kN * kN - 1, T, r.J);
    if (jlo == jhi) continue;  // one range covered the whole point tile: stored by its epilogue
    const int f = nt * kFB + f4 * 4;
    const int p = pt * kFB + tl;
    if (f >= r.Kg || p >= r.P) continue;
    const int tj = p % r.tx, pq = p / r.tx, ti = pq % r.ty, n = pq / r.ty;
    const int oy = ti * kM + q / kM, ox = tj * kM + q % kM;
    if (oy >= r.Ho || ox >= r.Wo) continue;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int j = jlo; j <= jhi; ++j) {
      const int slot = (sk_start(j, T, r.J) / (kN * kN) == pt) ? 0 : 1;  // its first range piece, else its last
      v += *reinterpret_cast<const f32x4*>(r.slab + ((static_cast<size_t>(j * r.n_ntiles + nt) * 2 + slot) * Q + q) *
                                                         (kFB * kFB) + tl * kFB + f4 * 4);
    }
    if (r.bias) v += *reinterpret_cast<const f32x4*>(r.bias + f);
    if (r.relu) v = f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
    *reinterpret_cast<f32x4*>(r.y + ((static_cast<size_t>(n) * r.Ho + oy) * r.Wo + ox) * r.K + f) = v;
  }
}

int device_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

unsigned grid_for(long n) {
  long g = (n + kT - 1) / kT;
  return static_cast<unsigned>(g > 65535 ? 65535 : (g < 1 ? 1 : g));
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
  // 49*groups independent GEMMs [P x C/g] x [C/g x K/g] as one grouped 1x1 "conv" over P pixels
  w.gemm = make_conv_plan(w.P, 1, 1, kN * kN * C, kN * kN * K, 1, 1, kN * kN * groups);
  return w;
}

bool wino_eligible(int F, int S, int C, int K, int groups) {
  return F == wino::kR && S == 1 && C % 4 == 0 && K % 4 == 0 && (C / groups) % 4 == 0 && (K / groups) % 4 == 0;
}

size_t wino_v_floats(const WinoPlan& w) { return static_cast<size_t>(w.P) * kN * kN * w.C; }
size_t wino_m_floats(const WinoPlan& w) { return static_cast<size_t>(w.P) * kN * kN * w.K; }

void wino_transform_weights_host(const WinoPlan& w, const float* w_kcff, std::vector<float>& u_kcff) {
  // U[(ab*groups + g)*Kg + k][c] = (G g_{k,c} G^T)[a][b], computed in fp64 then rounded once.
  const int Cg = w.C / w.groups, Kg = w.K / w.groups, R = wino::kR;
  u_kcff.assign(static_cast<size_t>(kN * kN) * w.K * Cg, 0.f);
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

hipError_t wino_input(const WinoPlan& w, const float* x, float* V, hipStream_t s, bool nt, bool scalar) {
  const long n = static_cast<long>(w.P) * w.C;
  if (n >= (1L << 31)) return hipErrorInvalidValue;
  const long g = (n + kT - 1) / kT;
  const unsigned gg = static_cast<unsigned>(g < (1 << 20) ? g : (1 << 20));
  if (w.C % 2 == 0 && !scalar) {  // 2 channels per thread
    const long g2 = (n / 2 + kT - 1) / kT;
    const unsigned gg2 = static_cast<unsigned>(g2 < (1 << 20) ? g2 : (1 << 20));
    if (nt)
      wino_in2_kernel<true><<<gg2, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
    else
      wino_in2_kernel<false><<<gg2, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
    return hipGetLastError();
  }
  if (nt)  // A/B: non-temporal V stores
    wino_in_kernel<true><<<gg, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
  else
    wino_in_kernel<false><<<gg, kT, 0, s>>>(x, V, w.N, w.Hq, w.Wq, w.C, w.ty, w.tx);
  return hipGetLastError();
}

hipError_t wino_input_pool(const WinoPlan& w, const float* c1, const WinoPoolGeom& pg, float* V, hipStream_t s) {
  const long n = static_cast<long>(w.P) * w.C;
  if (n >= (1L << 31) || static_cast<long>(w.N) * pg.H1 * pg.W1 * w.C >= (1L << 31)) return hipErrorInvalidValue;
  // every pooled window row must read conv1 rows inside the buffer: 0 <= 2*p1_lo - c1_lo and
  // 2*(p1_hi - 1) + 2 - c1_lo < H1 (checked on the host: the kernel does not bound-check rows)
  if (pg.p1_hi > pg.p1_lo && (2 * pg.p1_lo - pg.c1_lo < 0 || 2 * (pg.p1_hi - 1) + 2 - pg.c1_lo >= pg.H1))
    return hipErrorInvalidValue;
  WinoPoolArgs g{};
  g.N = w.N;
  g.Hq = w.Hq;
  g.Wq = w.Wq;
  g.C = w.C;
  g.ty = w.ty;
  g.tx = w.tx;
  g.H1 = pg.H1;
  g.W1 = pg.W1;
  g.Wp = pg.Wp;
  g.pad = pg.pad;
  g.q_lo = pg.q_lo;
  g.p1_lo = pg.p1_lo;
  g.p1_hi = pg.p1_hi;
  g.c1_lo = pg.c1_lo;
  if (w.C % kPoolCg || w.Wq > kPoolMaxWq) return hipErrorInvalidValue;
  const long gb = static_cast<long>(w.N) * w.ty * (w.C / kPoolCg);
  if (gb >= (1L << 31)) return hipErrorInvalidValue;
  wino_in_pool_kernel<<<static_cast<unsigned>(gb), kPoolThreads, 0, s>>>(c1, V, g);
  return hipGetLastError();
}

// two rounds of co-resident workgroups' worth of 9 x 64 x 64 fold slabs (~150 MB at 256 CUs)
size_t wino_split_ws_floats() { return static_cast<size_t>(4) * device_cus() * kM * kM * kFB * kFB; }

// Tail split: whole rounds of workgroups run as usual; the point tiles of the last, partial round
// are split S ways by transform point. A CU's throughput is the same with one resident workgroup as
// with two (128 images: 512 workgroups in 253 us, then the 160-workgroup tail in 122 us), so a
// round is one workgroup per CU. In units of one workgroup's whole-tile time the tail then costs
// ceil(S * tail / CUs) / S, plus ~0.09 per CU-round of slabs written and summed (a 147 KB slab
// round trip per split workgroup); S = 1 costs 1. S is the cheapest of 1..7 within the workspace:
// 3 at 128 images, 7 at 256 (16 tail workgroups), none at 300 (the tail round is 94 % full).
WinoSplit plan_wino_split(const WinoPlan& w, const Knobs& kn) {
  WinoSplit sp{0, 0, 1};
  const int n_ptiles = (w.P + kFB - 1) / kFB, per_pt = (w.K / w.groups + kFB - 1) / kFB * w.groups;  // WGs per point tile
  sp.pt_full = n_ptiles;
  if (kn.wino_split == 0 || (kn.wino_cfg & 15) != 7 || (kn.wino_prio & ~(257 | 512)) != 0) return sp;
  const long slots = device_cus();  // throughput rounds (see above)
  const long wgs = static_cast<long>(n_ptiles) * per_pt;
  const long full_rounds = wgs / slots;
  int pt_full = static_cast<int>(full_rounds * slots / per_pt / 8 * 8);  // whole XCD groups of 8 point tiles
  if (pt_full > n_ptiles) pt_full = n_ptiles;
  const int tail_pt = n_ptiles - pt_full;
  if (tail_pt == 0) return sp;
  const long tail_wgs = static_cast<long>((tail_pt + 7) / 8 * 8) * per_pt;
  const long cap = static_cast<long>(wino_split_ws_floats() / (kM * kM * kFB * kFB));  // slabs
  int best = 1;
  double best_cost = 1.0;
  for (int S = 2; S <= 7; ++S) {
    if (S * tail_wgs > cap) break;
    const double cost = static_cast<double>((S * tail_wgs + slots - 1) / slots) / S +
                        0.09 * static_cast<double>(S * tail_wgs) / static_cast<double>(slots);
    if (kn.wino_split == S || (kn.wino_split == 1 && cost < best_cost * 0.97)) {
      best = S;
      best_cost = cost;
      if (kn.wino_split == S) break;
    }
  }
  if (best < 2) return sp;
  sp.pt_full = pt_full;
  sp.tail_pt = tail_pt;
  sp.nsplit = best;
  return sp;
}

hipError_t wino_fused(const WinoPlan& w, const float* V, const float* U, const float* bias, float* y, bool relu,
                      hipStream_t s, const Knobs& kn, float* split_ws) {
  const int cfg = kn.wino_cfg, prio = kn.wino_prio, occ = kn.conv2_occ;
  const bool sf = (kn.fold_scalar & 2) != 0;
  FusedArgs a{};
  a.V = V;
  a.U = U;
  a.bias = bias;
  a.y = y;
  a.P = w.P;
  a.C = w.C;
  a.Cg = w.C / w.groups;
  a.Kg = w.K / w.groups;
  a.K = w.K;
  a.groups = w.groups;
  a.kpad = w.gemm.kpad;
  a.kpad_n = w.gemm.kpad_n;
  a.N = w.N;
  a.Ho = w.Ho;
  a.Wo = w.Wo;
  a.ty = w.ty;
  a.tx = w.tx;
  a.relu = relu ? 1 : 0;
  a.prio = prio;
  a.n_ptiles = (w.P + kFB - 1) / kFB;
  a.n_ntiles = (a.Kg + kFB - 1) / kFB;
  if (a.n_ntiles * kFB > a.kpad_n || a.Cg % 4) return hipErrorInvalidValue;
  {
    const long vb = static_cast<long>(w.P) * kN * kN * w.C * 4, ub = static_cast<long>(kN * kN) * w.groups * a.kpad_n * a.kpad * 4;
    const bool buf = !(prio & 512) && vb < (1L << 31) && ub < (1L << 31);  // prio bit 9: global_load_lds (A/B)
    a.vbytes = buf ? static_cast<int>(vb) : 0;
    a.ubytes = buf ? static_cast<int>(ub) : 0;
  }
  const bool xcd = (cfg & 2) != 0;
  if ((cfg & 8) && a.Cg % 48 == 0 && a.kpad == a.Cg && a.Kg % 32 == 0) {
    // 16x16 MFMA: bit0 set -> 64 tiles x 64 filters, 8 waves, 2 workgroups/CU; bit0 clear -> 64 tiles
    // x 128 filters, 16 waves, 1 workgroup/CU (a quarter fewer operand bytes per MAC)
    if (cfg & 1) return xcd ? launch_glds16<4, 2, true>(a, s) : launch_glds16<4, 2, false>(a, s);
    if (a.Kg % 128 == 0) return xcd ? launch_glds16<4, 4, true>(a, s) : launch_glds16<4, 4, false>(a, s);
  }
  if (cfg & 4) {
    // LDS-DMA ring: BK 48 (72 KiB, 2 workgroups/CU) or BK 32 (48 KiB, 3/CU)
    const int bk = (cfg & 1) ? 48 : 32;
    if (a.Cg % bk == 0 && a.kpad == a.Cg) {
      const dim3 grid((xcd ? (a.n_ptiles + 7) / 8 * 8 : a.n_ptiles) * a.n_ntiles, 1, w.groups);
      if (bk == 48 && xcd && kn.wino_sk > 0 && split_ws && w.groups == 1 && a.kpad == 96 && (prio & ~257) == 0) {
        // stream-K: J ranges of equal (point tile, point) work, kn.wino_sk workgroups per CU
        const int J = std::min(a.n_ptiles, device_cus() * kn.wino_sk / a.n_ntiles);
        if (J >= 1 && static_cast<size_t>(J) * a.n_ntiles * 2 * kM * kM * kFB * kFB <= wino_split_ws_floats()) {
          FusedArgs k = a;
          k.slab = split_ws;
          k.sk_groups = J;
          const size_t lds = occupancy_lds(3 * 2 * kFB * 48 * sizeof(float), occ);
          static const hipError_t attr = [] {
            for (const void* f : {reinterpret_cast<const void*>(wino_fused_sk_kernel<true, true>),
                                  reinterpret_cast<const void*>(wino_fused_sk_kernel<false, true>),
                                  reinterpret_cast<const void*>(wino_fused_sk_kernel<true, false>),
                                  reinterpret_cast<const void*>(wino_fused_sk_kernel<false, false>)}) {
              const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
              if (e != hipSuccess) return e;
            }
            return hipSuccess;
          }();
          if (attr != hipSuccess) return attr;
          const dim3 gk((J + 7) / 8 * 8 * a.n_ntiles);
          const bool il = (prio & 256) != 0;  // full point tiles on the interleaved-fold schedule
          if (sf)
            il ? wino_fused_sk_kernel<true, true><<<gk, 256, lds, s>>>(k) : wino_fused_sk_kernel<true, false><<<gk, 256, lds, s>>>(k);
          else
            il ? wino_fused_sk_kernel<false, true><<<gk, 256, lds, s>>>(k)
               : wino_fused_sk_kernel<false, false><<<gk, 256, lds, s>>>(k);
          hipError_t e = hipGetLastError();
          if (e != hipSuccess) return e;
          SkReduceArgs r{split_ws, bias, y, J, a.n_ptiles, a.n_ntiles, w.P, a.Kg, w.K, w.Ho, w.Wo, w.ty, w.tx,
                         relu ? 1 : 0};
          const long n = static_cast<long>(a.n_ptiles) * a.n_ntiles * kM * kM * kFB * (kFB / 4);
          wino_sk_reduce_kernel<<<grid_for(n), 256, 0, s>>>(r);
          return hipGetLastError();
        }
      }
      const WinoSplit sp = split_ws ? plan_wino_split(w, kn) : WinoSplit{a.n_ptiles, 0, 1};
      if (bk == 48 && xcd && sp.nsplit > 1 &&
          static_cast<size_t>(sp.nsplit) * ((sp.tail_pt + 7) / 8 * 8) * a.n_ntiles * w.groups * kM * kM * kFB * kFB <=
              wino_split_ws_floats()) {
        // whole rounds of point tiles as usual, then the tail tiles' 49 points split nsplit ways
        // over the CUs the tail round would leave idle, then the slab sum (deterministic order)
        if (sp.pt_full > 0) {
          FusedArgs f = a;
          f.n_ptiles = sp.pt_full;
          const dim3 gf(sp.pt_full * a.n_ntiles, 1, w.groups);
          const hipError_t e = ((prio & 256) && a.kpad == 96)
                                   ? (sf ? launch_glds<48, true, true, true>(f, gf, s, occ)
                                         : launch_glds<48, true, true, false>(f, gf, s, occ))
                                   : (sf ? launch_glds<48, true, false, true>(f, gf, s, occ)
                                         : launch_glds<48, true, false, false>(f, gf, s, occ));
          if (e != hipSuccess) return e;
        }
        FusedArgs t = a;
        t.n_ptiles = sp.tail_pt;
        t.pt_base = sp.pt_full;
        t.nsplit = sp.nsplit;
        t.slab = split_ws;
        const dim3 gt((sp.tail_pt + 7) / 8 * 8 * a.n_ntiles, sp.nsplit, w.groups);
        const hipError_t e = sf ? launch_glds<48, true, false, true>(t, gt, s, occ)
                                : launch_glds<48, true, false, false>(t, gt, s, occ);
        if (e != hipSuccess) return e;
        SplitReduceArgs r{split_ws, bias, y, sp.nsplit, sp.tail_pt, a.n_ntiles, sp.pt_full, w.groups,
                          w.P,      a.Kg, w.K, w.Ho,      w.Wo,       w.ty,     w.tx,     relu ? 1 : 0};
        const long n = static_cast<long>(w.groups) * sp.tail_pt * a.n_ntiles * kM * kM * kFB * (kFB / 4);
        wino_split_reduce_kernel<<<grid_for(n), 256, 0, s>>>(r);
        return hipGetLastError();
      }
      if (bk == 48 && xcd) {  // the interleaved fold needs exactly 2 K slices per point (C = 96)
        if ((prio & 256) && a.kpad == 96)
          return sf ? launch_glds<48, true, true, true>(a, grid, s, occ)
                    : launch_glds<48, true, true, false>(a, grid, s, occ);
        return sf ? launch_glds<48, true, false, true>(a, grid, s, occ)
                  : launch_glds<48, true, false, false>(a, grid, s, occ);
      }
      if (bk == 48) return launch_glds<48, false>(a, grid, s, occ);
      if (xcd) return launch_glds<32, true>(a, grid, s, occ);
      return launch_glds<32, false>(a, grid, s, occ);
    }
  }
  const int bk = (a.kpad % 48 == 0 && cfg & 1) ? 48 : 32;
  dim3 grid((xcd ? (a.n_ptiles + 7) / 8 * 8 : a.n_ptiles) * a.n_ntiles, 1, w.groups);
  if (bk == 48 && xcd)
    wino_fused_kernel<48, true><<<grid, 256, 0, s>>>(a);
  else if (bk == 48)
    wino_fused_kernel<48, false><<<grid, 256, 0, s>>>(a);
  else if (xcd)
    wino_fused_kernel<32, true><<<grid, 256, 0, s>>>(a);
  else
    wino_fused_kernel<32, false><<<grid, 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t wino_output(const WinoPlan& w, const float* Mt, const float* bias, float* y, bool relu, hipStream_t s) {
  const long n = static_cast<long>(w.P) * (w.K / 4);
  wino_out_kernel<<<grid_for(n), kT, 0, s>>>(Mt, bias, y, w.N, w.Ho, w.Wo, w.K, w.ty, w.tx, relu ? 1 : 0);
  return hipGetLastError();
}

}  // namespace anx::hip
