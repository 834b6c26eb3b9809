// bf16 path for the full-AlexNet extension (BASELINE.json config "Full AlexNet Conv1-5 + FC6-8
// bf16"): implicit-GEMM convolution / fully-connected layers on v_mfma_f32_32x32x16_bf16 with fp32
// accumulation, fused bias + ReLU, bf16 NHWC activations; bf16 max-pool and max-pool+LRN that write
// straight into the next layer's zero-bordered window.
//
// Same structure as the fp32 kernel (conv_mfma.hip): 4 waves x (TM*32) x (TN*32) accumulators,
// LDS-staged K slices (BK = 64 bf16 here) with a lane-contiguous k permutation — for the bf16 MFMA
// lane (r, h) at k-step s holds A[r][16s + 8h + j], j = 0..7, i.e. one ds_read_b128 per operand
// per MFMA. Row stride BK+8 elements = 144 B (odd multiple of 16 B): conflict-free b128 reads.
// An FC layer is the 1x1 case: N images are N "pixels" of a 1x1 input with C = in_features.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <type_traits>
#include <vector>

#include "anx/bf16_ops.hpp"
#include "anx/hip_sync.hpp"
#include "anx/lrn_math.hpp"

namespace anx::hip {
namespace {

using bf16 = __bf16;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
// taps8 gathers start at any bf16 (2-byte alignment); still one global_load_dwordx4 on gfx950.
using u32x4u = __attribute__((ext_vector_type(4), aligned(2))) unsigned;

constexpr int kThreads = 256;
constexpr int kBK = 64;
constexpr int kLDA = kBK + 8;

struct ArgsB {
  const bf16* x;
  const bf16* w;
  const int* koff;
  const float* bias;
  void* out;
  int M, HoWo, Wo, Hp, Wp, C, S, Cg, Kg, kpad, kpad_n, ktiles;
  int Hb, Wb, Cb, h_off, w_off, c_off, relu, n_ntiles;
  int kt_per;           // K tiles per blockIdx.y slice (split-K; = ktiles when not split)
  size_t split_stride;  // output elements between split-K partial slabs
};

template <int BM, int BN, int WAVES_M, int WAVES_N, bool VEC8, typename OutT>
__global__ void __launch_bounds__(kThreads, VEC8 ? 3 : 2) conv_bf16_kernel(ArgsB a) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 32, TN = WN / 32;
  constexpr int A_UNITS = VEC8 ? kBK / 8 : kBK;  // per staged row
  constexpr int A_LOADS = BM * A_UNITS / kThreads;
  constexpr int B_LOADS = BN * (kBK / 8) / kThreads;
  constexpr int A_STEP = kThreads / A_UNITS, B_STEP = kThreads / (kBK / 8);
  static_assert(A_LOADS * kThreads == BM * A_UNITS && B_LOADS * kThreads == BN * (kBK / 8), "tile split");
  extern __shared__ __attribute__((aligned(16))) bf16 lds_b[];
  bf16* As = lds_b;
  bf16* Bs = lds_b + BM * kLDA;
  int* koff_s = reinterpret_cast<int*>(lds_b + (BM + BN) * kLDA);
  int* ooff_s = koff_s + a.kpad;  // output offset per tile row (-1 past M), from the prologue

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int wm = wave / WAVES_N, wn = wave % WAVES_N, g = blockIdx.z;
  const int mt = blockIdx.x / a.n_ntiles, nt = blockIdx.x - mt * a.n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const bf16* x = a.x + g * a.Cg;
  const bf16* wg = a.w + static_cast<size_t>(g) * a.kpad_n * a.kpad;
  for (int i = tid; i < a.kpad; i += kThreads) koff_s[i] = a.koff[i];
  const int au = tid % A_UNITS;
  int org[A_LOADS];
  unsigned ok = 0;
#pragma unroll
  for (int j = 0; j < A_LOADS; ++j) {
    const int row = tid / A_UNITS + j * A_STEP;
    const int m = m0 + row;
    int o = 0, oo = -1;
    if (m < a.M) {
      const int n = m / a.HoWo, r = m - n * a.HoWo, oy = r / a.Wo, ox = r - oy * a.Wo;
      o = ((n * a.Hp + oy * a.S) * a.Wp + ox * a.S) * a.C;
      oo = ((n * a.Hb + oy + a.h_off) * a.Wb + ox + a.w_off) * a.Cb + a.c_off;
    }
    if (au == 0) ooff_s[row] = oo;
    org[j] = o;
    ok |= (m < a.M ? 1u : 0u) << j;
  }
  const int bu = tid % (kBK / 8);
  const bf16* bsrc = wg + static_cast<size_t>(n0 + tid / (kBK / 8)) * a.kpad + bu * 8;
  __syncthreads();

  using AReg = typename std::conditional<VEC8, u32x4, bf16>::type;
  AReg ra[A_LOADS];
  u32x4 rb[B_LOADS];
  bool kok = true;
  auto load = [&](int kt) {
    const int kb = kt * kBK;
    const int ko_raw = koff_s[kb + (VEC8 ? au * 8 : au)];
    kok = ko_raw >= 0;
    const int ko = kok ? ko_raw : 0;
#pragma unroll
    for (int j = 0; j < A_LOADS; ++j) {
      if constexpr (VEC8)
        ra[j] = *reinterpret_cast<const u32x4u*>(x + org[j] + ko);
      else
        ra[j] = x[org[j] + ko];
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j)
      rb[j] = *reinterpret_cast<const u32x4*>(bsrc + static_cast<size_t>(j) * B_STEP * a.kpad + kb);
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < A_LOADS; ++j) {
      const int row = tid / A_UNITS + j * A_STEP;
      const bool v = kok && ((ok >> j) & 1u);
      if constexpr (VEC8)
        *reinterpret_cast<u32x4*>(As + row * kLDA + au * 8) = v ? ra[j] : u32x4{0u, 0u, 0u, 0u};
      else
        As[row * kLDA + au] = v ? ra[j] : static_cast<bf16>(0.f);
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j)
      *reinterpret_cast<u32x4*>(Bs + (tid / (kBK / 8) + j * B_STEP) * kLDA + bu * 8) = rb[j];
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  const int r = lane & 31, h = lane >> 5;
  const bf16* ard = As + (wm * WM + r) * kLDA + h * 8;
  const bf16* brd = Bs + (wn * WN + r) * kLDA + h * 8;
  const int kt0 = blockIdx.y * a.kt_per, kt1 = min(a.ktiles, kt0 + a.kt_per);
  if (kt0 < kt1) {
    load(kt0);
    store();
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    if (kt + 1 < kt1) load(kt + 1);
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ard + i * 32 * kLDA + s * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(brd + j * 32 * kLDA + s * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (kt + 1 < kt1) {
      store();
      __syncthreads();
    }
  }
  OutT* out = static_cast<OutT*>(a.out) + blockIdx.y * a.split_stride + g * a.Kg;
  using i32x4 = __attribute__((ext_vector_type(4))) int;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    i32x4 oo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) oo[q] = *reinterpret_cast<const i32x4*>(ooff_s + wm * WM + i * 32 + 8 * q + 4 * h);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int f = n0 + wn * WN + j * 32 + r;
      if (f >= a.Kg) continue;
      const float bv = a.bias ? a.bias[g * a.Kg + f] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = oo[e >> 2][e & 3];
        if (o < 0) continue;
        float v = acc[i][j][e] + bv;
        if (a.relu) v = fmaxf(v, 0.f);
        out[o + f] = static_cast<OutT>(v);
      }
    }
  }
}

// ---- LDS-DMA ring variant of the 128x128 vec8 kernel (conv2-5, FC) ----
// The register-staged kernel above pays two __syncthreads per K tile and drains its global loads
// at each (cdna_hip_programming.md §5: the 2-barrier structure's ceiling). Here operand tiles go
// global -> LDS by global_load_lds_dwordx4 (per-lane gather addresses: A row = output pixel window
// origin + koff of the K slice's tap, B row = packed filter) into an NST-deep ring retired by a
// counted vmcnt and ONE raw barrier per K tile (the fp32 Winograd GEMM's structure, winograd.hip).
// LDS rows are 64 bf16 = 8 16-B units, unit u of row r stored at u ^ ((r >> 1) & 7): the 16 rows
// of every ds_read_b128 lane group hit 16 distinct bank quads. No zero-masking: rows past M point
// at pixel 0 and are never stored; K padding (koff -1 -> 0) meets zero-packed weights.
using lds_b16 = __attribute__((address_space(3))) bf16;
__device__ __forceinline__ void glds16_b(const bf16* g, lds_b16* l) { __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// WMW waves along M (BM = 64*WMW pixels) x 2 along N (BN = 128 filters), 64x64 per wave.
template <int NST, int WMW, typename OutT>
__global__ void __launch_bounds__(128 * WMW) conv_bf16_glds_kernel(ArgsB a) {
  constexpr int NT = 128 * WMW;                                      // threads
  constexpr int BM = 64 * WMW, BN = 128, TM = 2, TN = 2, BKU = kBK / 8;  // 8 units per row
  constexpr int ATILE = BM * kBK, BTILE = BN * kBK;                  // bf16 per operand tile
  constexpr int STAGE = ATILE + BTILE;
  constexpr int NA = BM * BKU / NT, NB = BN * BKU / NT;              // DMA per thread per operand
  static_assert(NA * NT == BM * BKU && NB * NT == BN * BKU && NB >= 1, "tile split");
  constexpr int RPJ = NT / 8;                                        // rows per DMA round
  extern __shared__ __attribute__((aligned(16))) bf16 lds_b[];
  int* koff_s = reinterpret_cast<int*>(lds_b + NST * STAGE);
  int* ooff_s = koff_s + a.kpad;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int wm = wave >> 1, wn = wave & 1, g = blockIdx.z;
  const int mt = blockIdx.x / a.n_ntiles, nt = blockIdx.x - mt * a.n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const bf16* x = a.x + g * a.Cg;
  const bf16* wg = a.w + static_cast<size_t>(g) * a.kpad_n * a.kpad;
  for (int i = tid; i < a.kpad; i += NT) koff_s[i] = a.koff[i];
  // DMA slot S = j*NT + tid holds row S/8 = j*RPJ + tid/8 (RPJ % 16 == 0), physical unit tid%8 =
  // logical unit u of that row
  const int u = (tid & 7) ^ ((tid >> 4) & 7);
  int aorg[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int m = m0 + j * RPJ + (tid >> 3);
    aorg[j] = 0;
    if (m < a.M) {
      const int n = m / a.HoWo, r = m - n * a.HoWo, oy = r / a.Wo, ox = r - oy * a.Wo;
      aorg[j] = ((n * a.Hp + oy * a.S) * a.Wp + ox * a.S) * a.C;
    }
  }
  if (tid < BM) {
    const int m = m0 + tid;
    int oo = -1;
    if (m < a.M) {
      const int n = m / a.HoWo, r = m - n * a.HoWo, oy = r / a.Wo, ox = r - oy * a.Wo;
      oo = ((n * a.Hb + oy + a.h_off) * a.Wb + ox + a.w_off) * a.Cb + a.c_off;
    }
    ooff_s[tid] = oo;
  }
  const bf16* bsrc = wg + static_cast<size_t>(n0 + (tid >> 3)) * a.kpad + u * 8;
  __syncthreads();  // koff_s / ooff_s visible
  lds_b16* lds3 = (lds_b16*)(lds_b);
  const int kt0 = blockIdx.y * a.kt_per, kt1 = min(a.ktiles, kt0 + a.kt_per);
  const int total = kt1 > kt0 ? kt1 - kt0 : 0;
  auto issue = [&](int it) {
    const int kb = (kt0 + it) * kBK;
    const int kr = koff_s[kb + u * 8];
    const int ko = kr >= 0 ? kr : 0;
    lds_b16* st = lds3 + (it % NST) * STAGE;
#pragma unroll
    for (int j = 0; j < NA; ++j) glds16_b(x + aorg[j] + ko, st + (j * NT + wave * 64) * 8);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      glds16_b(bsrc + static_cast<size_t>(j) * RPJ * a.kpad + kb, st + ATILE + (j * NT + wave * 64) * 8);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  const int r = lane & 31, h = lane >> 5;
  int arow[TM], brow[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) arow[i] = wm * 64 + i * 32 + r;
#pragma unroll
  for (int j = 0; j < TN; ++j) brow[j] = wn * 64 + j * 32 + r;
#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < total) issue(i);
  for (int it = 0; it < total; ++it) {
    if (it + NST - 2 < total)
      lds_barrier<(NA + NB) * (NST - 2)>();  // slice it landed for every wave; slot (it-1) % NST is free
    else
      lds_barrier<0>();
    asm volatile("" ::: "memory");
    if (it + NST - 1 < total) issue(it + NST - 1);
    const bf16* base = lds_b + (it % NST) * STAGE;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(base + arow[i] * kBK + (((2 * s + h) ^ ((arow[i] >> 1) & 7)) * 8));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(base + ATILE + brow[j] * kBK + (((2 * s + h) ^ ((brow[j] >> 1) & 7)) * 8));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  OutT* out = static_cast<OutT*>(a.out) + blockIdx.y * a.split_stride + g * a.Kg;
  using i32x4 = __attribute__((ext_vector_type(4))) int;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    i32x4 oo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) oo[q] = *reinterpret_cast<const i32x4*>(ooff_s + wm * 64 + i * 32 + 8 * q + 4 * h);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int f = n0 + wn * 64 + j * 32 + r;
      if (f >= a.Kg) continue;
      const float bv = a.bias ? a.bias[g * a.Kg + f] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = oo[e >> 2][e & 3];
        if (o < 0) continue;
        float v = acc[i][j][e] + bv;
        if (a.relu) v = fmaxf(v, 0.f);
        out[o + f] = static_cast<OutT>(v);
      }
    }
  }
}

// ---- bf16 max-pool (8 channels per thread) and max-pool + LRN (fp32 math) ----
__global__ void __launch_bounds__(256) pool_bf16_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                        int F, int S, int Ho, int Wo, OutViewB o) {
  const int C8 = C / 8;
  const long total = static_cast<long>(N) * Ho * Wo * C8;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(i % C8);
    long q = i / C8;
    const int ox = static_cast<int>(q % Wo);
    q /= Wo;
    const int oy = static_cast<int>(q % Ho), n = static_cast<int>(q / Ho);
    float m[8];
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int fh = 0; fh < F; ++fh)
      for (int fw = 0; fw < F; ++fw) {
        const int iy = oy * S + fh, ix = ox * S + fw;
        if (iy >= H || ix >= W) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((static_cast<size_t>(n) * H + iy) * W + ix) * C + c8 * 8);
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], static_cast<float>(v[e]));
      }
    bf16x8 r;
    for (int e = 0; e < 8; ++e) r[e] = static_cast<bf16>(m[e]);
    *reinterpret_cast<bf16x8*>(o.base + (static_cast<size_t>(n * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) * o.Cb +
                               o.c_off + c8 * 8) = r;
  }
}

// Workgroup = (n, output row oy): the F input rows S*oy .. S*oy+F-1 are contiguous; each thread
// takes the column max over them for (column, 8 channels) pairs (16-B loads), stages it in LDS, then
// writes the Wo horizontal maxima as 16-B stores. Each input row is fetched by at most
// ceil(F / S) workgroups instead of each input pixel by ~(F / S)^2 output threads.
__global__ void __launch_bounds__(256) pool_rows_bf16_kernel(const bf16* __restrict__ x, int H, int W, int C, int F,
                                                             int S, int Ho, int Wo, OutViewB o) {
  extern __shared__ __attribute__((aligned(16))) bf16 colmax[];  // [W][C]
  const int oy = blockIdx.x, n = blockIdx.y, C8 = C / 8;
  const int y0 = oy * S, fh = min(F, H - y0);
  const bf16* src = x + (static_cast<size_t>(n) * H + y0) * W * C;
  for (int q = threadIdx.x; q < W * C8; q += 256) {  // q = column * C8 + chunk
    bf16x8 m = *reinterpret_cast<const bf16x8*>(src + q * 8);
    for (int r = 1; r < fh; ++r) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + static_cast<size_t>(r) * W * C + q * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = static_cast<bf16>(fmaxf(static_cast<float>(m[e]), static_cast<float>(v[e])));
    }
    *reinterpret_cast<bf16x8*>(colmax + q * 8) = m;
  }
  __syncthreads();
  bf16* dst = o.base + (static_cast<size_t>(n * o.Hb + oy + o.h_off) * o.Wb + o.w_off) * o.Cb + o.c_off;
  for (int q = threadIdx.x; q < Wo * C8; q += 256) {
    const int ox = q / C8, c8 = q - ox * C8, x0 = ox * S, fw = min(F, W - x0);
    bf16x8 m = *reinterpret_cast<const bf16x8*>(colmax + (x0 * C8 + c8) * 8);
    for (int c = 1; c < fw; ++c) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(colmax + ((x0 + c) * C8 + c8) * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = static_cast<bf16>(fmaxf(static_cast<float>(m[e]), static_cast<float>(v[e])));
    }
    *reinterpret_cast<bf16x8*>(dst + static_cast<size_t>(ox) * o.Cb + c8 * 8) = m;
  }
}

// One workgroup = PP output pixels x C channels; 8 channels per thread (16-B bf16 loads/stores).
// Pass 1 pools into LDS as fp32, pass 2 applies LRN from LDS: own 8 channels by two ds_read_b128,
// the +-2 neighbours by two ds_read_b64 (size-5 window), fp32 math, one bf16x8 store.
__global__ void __launch_bounds__(256) pool_lrn_bf16_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                            int F, int S, int Ho, int Wo, int PP, int size, float a,
                                                            float beta, float k, OutViewB o) {
  using f32x4 = __attribute__((ext_vector_type(4))) float;
  using f32x2 = __attribute__((ext_vector_type(2))) float;
  extern __shared__ __attribute__((aligned(16))) float pooled[];  // [PP][C]
  const int C8 = C / 8;
  const long P = static_cast<long>(N) * Ho * Wo, p0 = static_cast<long>(blockIdx.x) * PP;
  for (int t = threadIdx.x; t < PP * C8; t += blockDim.x) {
    const int pl = t / C8, c0 = (t - pl * C8) * 8;
    const long p = p0 + pl;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = p < P ? -INFINITY : 0.f;
    if (p < P) {
      const int ox = static_cast<int>(p % Wo);
      const long q = p / Wo;
      const int oy = static_cast<int>(q % Ho), n = static_cast<int>(q / Ho);
      for (int fh = 0; fh < F; ++fh) {
        const int iy = oy * S + fh;
        if (iy >= H) break;
        for (int fw = 0; fw < F; ++fw) {
          const int ix = ox * S + fw;
          if (ix >= W) break;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((static_cast<size_t>(n) * H + iy) * W + ix) * C + c0);
#pragma unroll
          for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], static_cast<float>(v[e]));
        }
      }
    }
    *reinterpret_cast<f32x4*>(pooled + pl * C + c0) = f32x4{m[0], m[1], m[2], m[3]};
    *reinterpret_cast<f32x4*>(pooled + pl * C + c0 + 4) = f32x4{m[4], m[5], m[6], m[7]};
  }
  __syncthreads();
  const int half = size / 2;
  for (int t = threadIdx.x; t < PP * C8; t += blockDim.x) {
    const int pl = t / C8, c0 = (t - pl * C8) * 8;
    const long p = p0 + pl;
    if (p >= P) continue;
    const float* row = pooled + pl * C;
    bf16x8 r;
    if (half == 2) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(row + c0), hi = *reinterpret_cast<const f32x4*>(row + c0 + 4);
      const f32x2 lf = c0 >= 2 ? *reinterpret_cast<const f32x2*>(row + c0 - 2) : f32x2{0.f, 0.f};
      const f32x2 rt = c0 + 8 < C ? *reinterpret_cast<const f32x2*>(row + c0 + 8) : f32x2{0.f, 0.f};
      const float w[12] = {lf.x, lf.y, lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w, rt.x, rt.y};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s2 = 0.f;
#pragma unroll
        for (int u = e; u < e + 5; ++u) s2 = fmaf(w[u], w[u], s2);
        r[e] = static_cast<bf16>(w[e + 2] * lrn_scale(s2, k, a, beta));
      }
    } else {
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        float s2 = 0.f;
        for (int j = c - half < 0 ? 0 : c - half; j <= (c + half >= C ? C - 1 : c + half); ++j)
          s2 = fmaf(row[j], row[j], s2);
        r[e] = static_cast<bf16>(row[c] * lrn_scale(s2, k, a, beta));
      }
    }
    const int ox = static_cast<int>(p % Wo);
    const long q = p / Wo;
    const int oy = static_cast<int>(q % Ho), n = static_cast<int>(q / Ho);
    *reinterpret_cast<bf16x8*>(o.base + (static_cast<size_t>(n * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) * o.Cb +
                               o.c_off + c0) = r;
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    y[i] = static_cast<bf16>(x[i]);
}

// pool + LRN for C = 256, size 5 (Conv2 -> Pool2 -> LRN2 of the full model). A half-wave owns one
// output pixel, 8 channels per lane (16-B loads and stores), and a wave walks U pixel pairs per
// step with all 9U loads in flight (one wave per 4-channel pixel was latency-bound: 74 us at 256
// images for 124 MB). LRN neighbours c-2, c-1 / c+8, c+9 come from the adjacent lanes' maxima by
// ds_bpermute, zero past each pixel's channel ends. Same maxima and the same ascending 5-term sums
// of squares as pool_lrn_bf16_kernel: bit-identical, without the LDS tile.
template <int F, int U>
__global__ void __launch_bounds__(256) pool_lrn256_bf16_kernel(const bf16* __restrict__ x, int P, int H, int W,
                                                               int S, int Ho, int Wo, float a, float beta, float k,
                                                               OutViewB o) {
  constexpr int C = 256;
  const int lane = threadIdx.x & 63, half = lane >> 5, cl = lane & 31;
  const int nw = gridDim.x * 4;
  for (int base = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 * U; base < P; base += nw * 2 * U) {  // wave-uniform
    float m[U][8];
    int pix[U];
    // every window load unconditional (clamped to a valid pixel, masked to -inf when outside): a
    // load inside a branch made the compiler wait for it at the join, one load in flight per wave
    bf16x8 wv[U][F * F];
    bool wok[U][F * F];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = base + 2 * u + half;
      pix[u] = p;
      const int pc = min(p, P - 1);
      const int ox = pc % Wo, q = pc / Wo, oy = q % Ho, n = q / Ho;
#pragma unroll
      for (int fh = 0; fh < F; ++fh) {
        const int iy = oy * S + fh;
#pragma unroll
        for (int fw = 0; fw < F; ++fw) {
          const int ix = ox * S + fw;
          wok[u][fh * F + fw] = iy < H && ix < W;
          wv[u][fh * F + fw] = *reinterpret_cast<const bf16x8*>(
              x + ((static_cast<size_t>(n) * H + min(iy, H - 1)) * W + min(ix, W - 1)) * C + cl * 8);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < 8; ++e) m[u][e] = -INFINITY;
#pragma unroll
      for (int t = 0; t < F * F; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) m[u][e] = fmaxf(m[u][e], wok[u][t] ? static_cast<float>(wv[u][t][e]) : -INFINITY);
    }
    const int left = ((lane + 63) & 63) * 4, right = ((lane + 1) & 63) * 4;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float l0 = __int_as_float(__builtin_amdgcn_ds_bpermute(left, __float_as_int(m[u][6])));
      float l1 = __int_as_float(__builtin_amdgcn_ds_bpermute(left, __float_as_int(m[u][7])));
      float r0 = __int_as_float(__builtin_amdgcn_ds_bpermute(right, __float_as_int(m[u][0])));
      float r1 = __int_as_float(__builtin_amdgcn_ds_bpermute(right, __float_as_int(m[u][1])));
      if (cl == 0) l0 = l1 = 0.f;
      if (cl == 31) r0 = r1 = 0.f;
      const int p = pix[u];
      if (p >= P) continue;
      const float w[12] = {l0, l1, m[u][0], m[u][1], m[u][2], m[u][3], m[u][4], m[u][5], m[u][6], m[u][7], r0, r1};
      bf16x8 r;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s2 = 0.f;
#pragma unroll
        for (int t = e; t < e + 5; ++t) s2 = fmaf(w[t], w[t], s2);
        r[e] = static_cast<bf16>(w[e + 2] * lrn_scale(s2, k, a, beta));
      }
      const int ox = p % Wo, q = p / Wo, oy = q % Ho, n = q / Ho;
      *reinterpret_cast<bf16x8*>(o.base + (static_cast<size_t>(n * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) * o.Cb +
                                 o.c_off + cl * 8) = r;
    }
  }
}

// Workgroup = (n, i): image rows 4i..4i+3 are one contiguous run of 4 W x 3 floats (one coalesced
// dword pass into LDS), and output row (n, i) — Wo pixels x 48 bf16 — is contiguous and 16-B
// aligned (Wo x 96 B): one 16-B store per 8 outputs, each gathered from LDS. (Thread-per-(pixel,
// polyphase row) with 12 scalar loads moved 238 MB in 54 us at 256 images.)
__global__ void __launch_bounds__(256) s2d4_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, int H, int W,
                                                        int Ho, int Wo) {
  extern __shared__ float rows[];  // [4][W * 3] from rows + mis (+ 8 floats of alignment slack)
  const int i = blockIdx.x, n = blockIdx.y, RW = W * 3;
  const int nrows = min(4, H - 4 * i);
  const size_t off = (static_cast<size_t>(n) * H + 4 * i) * RW;  // first float of the row group
  // 16-B loads from the 16-B aligned float at or below x + off (x may be an interior pointer of a
  // larger batch: the granule then still lies inside that allocation), stored as 16-B LDS writes at
  // the same alignment: LDS float p holds source float off - mis + p, so the image starts at rows + mis
  const int mis = static_cast<int>((reinterpret_cast<uintptr_t>(x + off) >> 2) & 3), nval = nrows * RW;
  const float4* src4 = reinterpret_cast<const float4*>(x + (off - mis));
  const int n4 = (mis + nval + 3) >> 2;
  for (int t = threadIdx.x; t < n4; t += 256) reinterpret_cast<float4*>(rows)[t] = src4[t];
  if (nval < 4 * RW) {  // the last row group: rows past the image are zero (block-uniform branch)
    __syncthreads();    // after the vector writes, whose last vector may reach past nval
    for (int t = nval + threadIdx.x; t < 4 * RW; t += 256) rows[mis + t] = 0.f;
  }
  __syncthreads();
  const float* rowsv = rows + mis;
  bf16* dst = y + (static_cast<size_t>(n) * Ho + i) * Wo * 48;
  for (int c = threadIdx.x; c < Wo * 6; c += 256) {  // 8 outputs per chunk, 6 chunks per pixel
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = c * 8 + e, j = q / 48, r = q - j * 48, rh = r / 12, rw = (r - rh * 12) / 3, ch = r - rh * 12 - rw * 3;
      const int col = 4 * j + rw;
      v[e] = static_cast<bf16>(col < W ? rowsv[rh * RW + col * 3 + ch] : 0.f);
    }
    *reinterpret_cast<bf16x8*>(dst + c * 8) = v;
  }
}


struct VariantB {
  int BM, BN;
  bool vec8;
};
constexpr VariantB kVB[] = {{128, 128, true}, {128, 96, false}, {64, 64, true},
                            {64, 64, false},  {128, 128, false}, {128, 96, true}};

unsigned grid1d(long n) {
  long g = (n + 255) / 256;
  return static_cast<unsigned>(g > 65535 ? 65535 : (g < 1 ? 1 : g));
}

}  // namespace

ConvPlanB make_conv_plan_bf16(int N, int Hp, int Wp, int C, int K, int F, int S, int groups) {
  ConvPlanB p{};
  p.N = N;
  p.Hp = Hp;
  p.Wp = Wp;
  p.C = C;
  p.K = K;
  p.F = F;
  p.S = S;
  p.groups = groups;
  p.Ho = conv_out_dim(Hp, F, S, 0);
  p.Wo = conv_out_dim(Wp, F, S, 0);
  p.Cg = C / groups;
  p.Kg = K / groups;
  p.kdim = F * F * p.Cg;
  p.vec8 = (p.Cg % 8 == 0 && C % 8 == 0) ? 1 : 0;
  p.taps8 = (!p.vec8 && groups == 1 && F * C >= 8) ? 1 : 0;
  if (p.taps8) {
    p.kdim = F * 8 * ((F * C + 7) / 8);
    p.vec8 = 1;
  }
  p.kpad = (p.kdim + kBK - 1) / kBK * kBK;
  const long M = static_cast<long>(N) * p.Ho * p.Wo;
  // 64x64 tiles below this many outputs (ANX_BF16_SMALL_MK overrides; A/B knob for wave quantization)
  static const long small_mk = [] {
    const char* e = std::getenv("ANX_BF16_SMALL_MK");
    return e ? std::atol(e) : 256L * 128 * 128;
  }();
  const bool small = M * K < small_mk;
  const bool fc = Hp == 1 && Wp == 1 && F == 1;  // fully-connected layer: 128x128 tiles + split-K
  if (fc && p.vec8) p.variant = 0;
  else if (p.Kg == 96 && !small) p.variant = p.vec8 ? 5 : 1;
  else if (small) p.variant = p.vec8 ? 2 : 3;
  else p.variant = p.vec8 ? 0 : 4;
  p.kpad_n = (p.Kg + kVB[p.variant].BN - 1) / kVB[p.variant].BN * kVB[p.variant].BN;
  return p;
}

size_t packed_weight_elems_bf16(const ConvPlanB& p) { return static_cast<size_t>(p.groups) * p.kpad_n * p.kpad; }

void pack_conv_weights_bf16(const ConvPlanB& p, const float* w_kcff, std::vector<uint16_t>& packed,
                            std::vector<int>& koff) {
  packed.assign(packed_weight_elems_bf16(p), 0);
  koff.assign(p.kpad, -1);
  if (p.taps8) {  // same unit scheme as the fp32 taps4 packing (conv_mfma.hip), 8 elements per unit
    const int L = p.F * p.C, U = (L + 7) / 8;
    for (int fh = 0; fh < p.F; ++fh)
      for (int u = 0; u < U; ++u)
        for (int e = 0; e < 8; ++e) {
          const int k = (fh * U + u) * 8 + e;
          const int f = (u < U - 1 ? 8 * u : L - 8) + e;
          koff[k] = fh * p.Wp * p.C + f;
          if (u == U - 1 && f < 8 * (U - 1)) continue;
          for (int n = 0; n < p.Kg; ++n)
            packed[static_cast<size_t>(n) * p.kpad + k] =
                f32_to_bf16_bits(w_kcff[((static_cast<size_t>(n) * p.C + f % p.C) * p.F + fh) * p.F + f / p.C]);
        }
    return;
  }
  for (int g = 0; g < p.groups; ++g)
    for (int n = 0; n < p.Kg; ++n)
      for (int fh = 0; fh < p.F; ++fh)
        for (int fw = 0; fw < p.F; ++fw)
          for (int c = 0; c < p.Cg; ++c) {
            const float v = w_kcff[((static_cast<size_t>(g * p.Kg + n) * p.Cg + c) * p.F + fh) * p.F + fw];
            packed[(static_cast<size_t>(g) * p.kpad_n + n) * p.kpad + (fh * p.F + fw) * p.Cg + c] = f32_to_bf16_bits(v);
          }
  for (int fh = 0; fh < p.F; ++fh)
    for (int fw = 0; fw < p.F; ++fw)
      for (int c = 0; c < p.Cg; ++c) koff[(fh * p.F + fw) * p.Cg + c] = (fh * p.Wp + fw) * p.C + c;
}

uint16_t f32_to_bf16_bits(float f) {  // round to nearest even, NaN kept NaN
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return static_cast<uint16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

hipError_t conv2d_bf16(const ConvPlanB& p, const void* x, const void* wpacked, const int* koff, const float* bias,
                       OutViewB out, float* out_f32, bool relu, hipStream_t s, SplitK split, int glds) {
  const long M = static_cast<long>(p.N) * p.Ho * p.Wo;
  if (M == 0) return hipSuccess;
  if (static_cast<long>(p.N) * p.Hp * p.Wp * p.C >= (1L << 31)) return hipErrorInvalidValue;
  const VariantB v = kVB[p.variant];
  ArgsB a{};
  a.x = static_cast<const bf16*>(x);
  a.w = static_cast<const bf16*>(wpacked);
  a.koff = koff;
  a.bias = bias;
  a.out = out_f32 ? static_cast<void*>(out_f32) : static_cast<void*>(out.base);
  a.M = static_cast<int>(M);
  a.HoWo = p.Ho * p.Wo;
  a.Wo = p.Wo;
  a.Hp = p.Hp;
  a.Wp = p.Wp;
  a.C = p.C;
  a.S = p.S;
  a.Cg = p.Cg;
  a.Kg = p.Kg;
  a.kpad = p.kpad;
  a.kpad_n = p.kpad_n;
  a.ktiles = p.kpad / kBK;
  a.Hb = out.Hb;
  a.Wb = out.Wb;
  a.Cb = out.Cb;
  a.h_off = out.h_off;
  a.w_off = out.w_off;
  a.c_off = out.c_off;
  a.relu = relu ? 1 : 0;
  a.n_ntiles = p.kpad_n / v.BN;
  const int ksplit = std::max(1, split.ksplit);
  a.kt_per = (a.ktiles + ksplit - 1) / ksplit;
  if (ksplit > 1) {  // fp32 partial slabs [ksplit][M][Kg] in split.ws, no bias/ReLU (splitk_reduce_bf16)
    if (p.groups != 1 || p.Ho != 1 || p.Wo != 1 || !split.ws) return hipErrorInvalidValue;
    out_f32 = split.ws;
    a.out = split.ws;
    a.bias = nullptr;
    a.relu = 0;
    a.Hb = a.Wb = 1;
    a.Cb = p.Kg;
    a.h_off = a.w_off = a.c_off = 0;
    a.split_stride = static_cast<size_t>(M) * p.Kg;
  }
  const dim3 grid(static_cast<unsigned>((M + v.BM - 1) / v.BM) * a.n_ntiles, ksplit, p.groups);
  const size_t lds = static_cast<size_t>(v.BM + v.BN) * kLDA * 2 + static_cast<size_t>(p.kpad + v.BM) * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
#define ANX_LAUNCH(BM, BN, WMW, WNW, V8)                                                              \
  do {                                                                                                \
    if (out_f32)                                                                                      \
      conv_bf16_kernel<BM, BN, WMW, WNW, V8, float><<<grid, kThreads, lds, s>>>(a);                   \
    else                                                                                              \
      conv_bf16_kernel<BM, BN, WMW, WNW, V8, bf16><<<grid, kThreads, lds, s>>>(a);                    \
  } while (0)
  if (p.variant == 0 && !p.taps8 && glds > 0) {
    // LDS-DMA ring: NST slots of (A|B) 128 x 64 bf16 tiles + the koff/ooff tables
    const int nst = glds == 2 ? 2 : 3;
    const size_t lds_r = static_cast<size_t>(nst) * 2 * 128 * kBK * 2 + static_cast<size_t>(p.kpad + 128) * 4;
    if (lds_r <= 160 * 1024) {
      // dynamic LDS above the 64 KiB default: opt every instantiation in once
      static const hipError_t attr = [] {
        const void* ks[] = {reinterpret_cast<const void*>(conv_bf16_glds_kernel<2, 2, float>),
                            reinterpret_cast<const void*>(conv_bf16_glds_kernel<2, 2, bf16>),
                            reinterpret_cast<const void*>(conv_bf16_glds_kernel<3, 2, float>),
                            reinterpret_cast<const void*>(conv_bf16_glds_kernel<3, 2, bf16>)};
        for (const void* k : ks) {
          const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
          if (e != hipSuccess) return e;
        }
        return hipSuccess;
      }();
      if (attr != hipSuccess) return attr;
      if (nst == 2 && out_f32)
        conv_bf16_glds_kernel<2, 2, float><<<grid, kThreads, lds_r, s>>>(a);
      else if (nst == 2)
        conv_bf16_glds_kernel<2, 2, bf16><<<grid, kThreads, lds_r, s>>>(a);
      else if (out_f32)
        conv_bf16_glds_kernel<3, 2, float><<<grid, kThreads, lds_r, s>>>(a);
      else
        conv_bf16_glds_kernel<3, 2, bf16><<<grid, kThreads, lds_r, s>>>(a);
      return hipGetLastError();
    }
  }
  switch (p.variant) {
    case 0: ANX_LAUNCH(128, 128, 2, 2, true); break;
    case 1: ANX_LAUNCH(128, 96, 4, 1, false); break;
    case 2: ANX_LAUNCH(64, 64, 2, 2, true); break;
    case 3: ANX_LAUNCH(64, 64, 2, 2, false); break;
    case 4: ANX_LAUNCH(128, 128, 2, 2, false); break;
    case 5: ANX_LAUNCH(128, 96, 4, 1, true); break;
    default: return hipErrorInvalidValue;
  }
#undef ANX_LAUNCH
  return hipGetLastError();
}

namespace {
// y[m][n] = act(sum_s ws[s][m][n] + bias[n]); 4 features per thread, bf16 (OutViewB) or fp32 out
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int ksplit, int M, int K,
                                                            const float* __restrict__ bias, int relu, OutViewB o,
                                                            float* __restrict__ out_f32) {
  using f32x4 = __attribute__((ext_vector_type(4))) float;
  const int K4 = K / 4;
  const long total = static_cast<long>(M) * K4;
  const size_t slab = static_cast<size_t>(M) * K;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int m = static_cast<int>(i / K4), n = static_cast<int>(i - static_cast<long>(m) * K4) * 4;
    f32x4 v = bias ? *reinterpret_cast<const f32x4*>(bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < ksplit; ++s) v += *reinterpret_cast<const f32x4*>(ws + s * slab + static_cast<size_t>(m) * K + n);
    if (relu) v = f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
    if (out_f32) {
      *reinterpret_cast<f32x4*>(out_f32 + static_cast<size_t>(m) * K + n) = v;
    } else {
      using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
      *reinterpret_cast<bf16x4*>(o.base + static_cast<size_t>(m) * o.Cb + o.c_off + n) =
          bf16x4{static_cast<bf16>(v.x), static_cast<bf16>(v.y), static_cast<bf16>(v.z), static_cast<bf16>(v.w)};
    }
  }
}
}  // namespace


int fc_split_k(const ConvPlanB& p) {
  if (p.Ho != 1 || p.Wo != 1 || p.groups != 1 || p.Kg % 4) return 1;
  const VariantB v = kVB[p.variant];
  const long tiles = (static_cast<long>(p.N) + v.BM - 1) / v.BM * (p.kpad_n / v.BN);
  const int ktiles = p.kpad / kBK;
  // ~256 workgroups (one per CU) but at least 4 K tiles per slice (guide: projection GEMM at M=256)
  const long want = (256 + tiles - 1) / tiles;
  return static_cast<int>(std::max<long>(1, std::min<long>(want, ktiles / 4)));
}

hipError_t splitk_reduce_bf16(const float* ws, int ksplit, int M, int K, const float* bias, bool relu, OutViewB out,
                              float* out_f32, hipStream_t s) {
  if (K % 4 || (!out_f32 && (out.Cb % 4 || out.c_off % 4))) return hipErrorInvalidValue;
  const long n = static_cast<long>(M) * (K / 4);
  if (n == 0) return hipSuccess;
  splitk_reduce_kernel<<<grid1d(n), 256, 0, s>>>(ws, ksplit, M, K, bias, relu ? 1 : 0, out, out_f32);
  return hipGetLastError();
}

hipError_t maxpool_bf16(const void* x, int N, int H, int W, int C, int F, int S, OutViewB out, hipStream_t s) {
  const int Ho = pool_out_dim(H, F, S), Wo = pool_out_dim(W, F, S);
  if (C % 8 || out.Cb % 8 || out.c_off % 8) return hipErrorInvalidValue;
  const long n = static_cast<long>(N) * Ho * Wo * (C / 8);
  if (n == 0) return hipSuccess;
  const size_t lds = static_cast<size_t>(W) * C * 2;
  if (lds <= 64 * 1024 && N <= 65535) {  // row kernel (max of bf16 values is exact: same result)
    pool_rows_bf16_kernel<<<dim3(Ho, N), 256, lds, s>>>(static_cast<const bf16*>(x), H, W, C, F, S, Ho, Wo, out);
    return hipGetLastError();
  }
  pool_bf16_kernel<<<grid1d(n), 256, 0, s>>>(static_cast<const bf16*>(x), N, H, W, C, F, S, Ho, Wo, out);
  return hipGetLastError();
}

hipError_t maxpool_lrn_bf16(const void* x, int N, int H, int W, int C, int F, int S, int size, float alpha,
                            float beta, float k, LrnMode mode, OutViewB out, hipStream_t s, int tile) {
  const int Ho = pool_out_dim(H, F, S), Wo = pool_out_dim(W, F, S);
  const long P = static_cast<long>(N) * Ho * Wo;
  if (P == 0) return hipSuccess;
  if (C % 8 || out.Cb % 8 || out.c_off % 8 || C > 8192) return hipErrorInvalidValue;
  const int PP = C >= 4096 ? 1 : 4096 / C;
  const float a = mode == LrnMode::DivN ? alpha / size : alpha;
  if (C == 256 && size == 5 && F == 3 && P < (1L << 31) && !tile) {
    constexpr int U = 2;  // pixel pairs per wave step
    const long waves = (P + 2 * U - 1) / (2 * U);
    pool_lrn256_bf16_kernel<3, U><<<static_cast<unsigned>((waves + 3) / 4), 256, 0, s>>>(
        static_cast<const bf16*>(x), static_cast<int>(P), H, W, S, Ho, Wo, a, beta, k, out);
    return hipGetLastError();
  }
  pool_lrn_bf16_kernel<<<static_cast<unsigned>((P + PP - 1) / PP), 256, PP * C * 4, s>>>(
      static_cast<const bf16*>(x), N, H, W, C, F, S, Ho, Wo, PP, size, a, beta, k, out);
  return hipGetLastError();
}

hipError_t f32_to_bf16(const float* x, void* y, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  f32_to_bf16_kernel<<<grid1d(static_cast<long>(n)), 256, 0, s>>>(x, static_cast<bf16*>(y), n);
  return hipGetLastError();
}

hipError_t f32_to_bf16_s2d4(const float* x, void* y, int N, int H, int W, hipStream_t s) {
  const int Ho = (H + 3) / 4, Wo = (W + 3) / 4;
  if (static_cast<long>(N) * Ho * Wo * 4 == 0) return hipSuccess;
  if (static_cast<long>(N) * H * W * 3 >= (1L << 31) || N > 65535 || W * 3 * 4 * 4 > 64 * 1024)
    return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(x) & 3) return hipErrorInvalidValue;
  s2d4_bf16_kernel<<<dim3(Ho, N), 256, (static_cast<size_t>(4) * W * 3 + 8) * 4, s>>>(x, static_cast<bf16*>(y), H, W,
                                                                                      Ho, Wo);
  return hipGetLastError();
}

}  // namespace anx::hip
