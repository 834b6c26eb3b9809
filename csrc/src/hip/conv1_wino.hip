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
//   1. conv1_wino_in_kernel   : image rows -> V [P][25][48] (P = N*ty*tx tiles; VALU, 16-B loads)
//   2. conv1_wino_gemm_kernel : for each of the 25 points ab, M_ab = V_ab[128 tiles x 48] .
//      U_ab[48 x 32 filters] on v_mfma_f32_32x32x2_f32 (exact fp32), folded straight into the 3x3
//      outputs (Y += A^T[i][a] A^T[j][b] M_ab; M never leaves registers), then bias + ReLU + NHWC
//      store through an OutView. Operand tiles go global -> LDS by LDS-DMA into an NST-deep ring
//      retired by a counted vmcnt and one raw barrier per slice (the Conv2 kernel's structure,
//      winograd.hip). 4 waves x 32 tiles share one 32-filter B tile: Conv1's 96 filters are exactly
//      3 workgroup columns (a 64-wide tile would waste a quarter of the MFMAs).
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
using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kT = 256;
constexpr int kPh = 4;                     // conv1 stride = polyphase factor
constexpr int kCh = kPh * kPh * 3;         // 48 polyphase channels
constexpr int kN5 = w33::kN;               // 5x5 transform tile
constexpr int kPts = kN5 * kN5;            // 25 transform points
constexpr int kPitch = w33::kM * kPh;      // 12 image rows/cols between tile origins
constexpr int kBM = 128, kBN = 32;         // tiles x filters per GEMM workgroup

// ---------------------------------------------------------------------------------------------
// Input transform. Thread = (tile p, phase row rh, 16-B unit j): at each of the 5x5 X' positions
// of the tile the 12 floats (rw, c) of phase row rh are 3 contiguous float4 units of one image row.
// Consecutive threads cover consecutive channels, so V rows (48 floats per (p, ab)) are written
// as whole 192-B runs.
template <bool NT>
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
        if constexpr (NT)
          __builtin_nontemporal_store(s, reinterpret_cast<f32x4*>(out + (a * kN5 + b) * kCh));
        else
          *reinterpret_cast<f32x4*>(out + (a * kN5 + b) * kCh) = s;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Batched GEMM + output transform.
struct AT33 {
  float v[w33::kM][w33::kN];
};
constexpr AT33 make_at33() {
  AT33 t{};
  for (int i = 0; i < w33::kM; ++i)
    for (int j = 0; j < w33::kN; ++j) t.v[i][j] = w33::kAT[i][j];
  return t;
}
__constant__ AT33 c_at33 = make_at33();  // indexed by the runtime point: scalar loads
// fold coefficients per point: coef[ab][i*3 + j] = A^T[i][a] * A^T[j][b] (the float product the
// runtime-indexed fold computes)
struct Coef33 {
  float v[kPts][9];
};
constexpr Coef33 make_coef33() {
  Coef33 t{};
  for (int ab = 0; ab < kPts; ++ab)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) t.v[ab][i * 3 + j] = w33::kAT[i][ab / kN5] * w33::kAT[j][ab % kN5];
  return t;
}
__constant__ Coef33 c_coef33 = make_coef33();

struct GemmArgs {
  const float* V;     // [P][25][48]
  const float* U;     // [25][K][48]
  const float* bias;  // [K]
  OutView out;        // conv1 output [N][H1][W1][K] (+ offsets)
  int P, K, H1, W1, ty, tx, relu, n_ptiles, n_ntiles;
  int probe;  // cost probes (wrong results; never set in production): bit0 no fold, bit1 no DMA
              // refill, bit2 no per-slice barrier (only with bit1), bit3 no epilogue stores;
              // bit4: s_setprio(1) around each slice's MFMAs (guide technique T5; on by default)
  int vbytes, ubytes;  // gemm16: > 0 = V / U byte sizes (< 2^31), operands by buffer_load ... lds
};

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
using f32x2 = __attribute__((ext_vector_type(2))) float;
template <bool SF>
__device__ __forceinline__ void fma2(f32x2& y, float c, float a0, float a1) {
  if constexpr (SF) {
    y.x = fmaf(c, a0, y.x);
    y.y = fmaf(c, a1, y.y);
  } else {
    y = __builtin_elementwise_fma(f32x2{c, c}, f32x2{a0, a1}, y);
  }
}

// LDS image per ring slot: [A: 128 rows x BK][B: 32 rows x BK], rows unpadded, the 16-B unit u of
// row r stored at u ^ ((r >> 2) & 3) (conflict-free ds_read_b128 fragment reads; the swizzle is
// applied to the DMA's per-lane global source address). The B tile needs fewer 1-KiB DMA
// instructions than A: wave w issues B instructions w, w+4, ...; waves with one more B DMA per slice
// wait with a larger counted vmcnt (two compile-time counts, picked by a wave-uniform branch).
template <int BK, int NST>
struct Ring {
  static constexpr int U4 = BK / 4;                  // 16-B units per row
  static constexpr int A_INS = kBM * U4 / 64;        // 1-KiB DMA instructions per A tile
  static constexpr int B_INS = kBN * U4 / 64;
  static constexpr int A_PW = A_INS / 4;             // per wave
  static constexpr int B_PW = (B_INS + 3) / 4;       // B slots per wave (the last may be empty)
  static constexpr int NS_LO = A_PW + B_INS / 4;     // DMA instructions per slice, waves >= B_INS % 4
  static constexpr int NS_HI = NS_LO + (B_INS % 4 ? 1 : 0);  // waves < B_INS % 4
  static constexpr int A_FL = kBM * BK, B_FL = kBN * BK;
  static constexpr int STAGE = A_FL + B_FL;
  static constexpr size_t kBytes = static_cast<size_t>(NST) * STAGE * sizeof(float);
  static_assert(A_PW * 4 == A_INS && B_INS * 64 == kBN * U4 && U4 % 4 == 0 && kCh % BK == 0, "tile shape");
  static_assert(kBytes <= 80 * 1024, "two workgroups per CU");
};

// s_waitcnt vmcnt(min(ahead, MAXA) * NSW): the DMAs of the `ahead` slices issued after the one
// being retired stay in flight (immediates only, so recurse over the possible depths).
template <int NSW, int MAXA>
__device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (MAXA > 0) {
    if (ahead >= MAXA) {
      wait_vmcnt<MAXA * NSW>();
      return;
    }
    wait_ahead<NSW, MAXA - 1>(ahead);
  } else {
    wait_vmcnt<0>();
  }
}

template <int BK, int NST, bool SF>
__global__ void __launch_bounds__(256, 2) conv1_wino_gemm_kernel(GemmArgs a) {
  using R = Ring<BK, NST>;
  constexpr int KS = kCh / BK;        // slices per transform point
  constexpr int TOTAL = kPts * KS;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  // XCD-aware order: the n_ntiles workgroups that read one V slab get equal blockIdx.x % 8, i.e.
  // one XCD under round-robin dispatch, so the slab comes from HBM/MALL once (speed only).
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles;
  const int pt = (jb / a.n_ntiles) * 8 + xcd;
  if (pt >= a.n_ptiles) return;  // whole workgroup: before any DMA or barrier
  const int p0 = pt * kBM, n0 = nt * kBN;

  int aoff[R::A_PW], boff[R::B_PW], bdst[R::B_PW];
#pragma unroll
  for (int j = 0; j < R::A_PW; ++j) {
    const int U = (j * 4 + wave) * 64 + lane;
    const int row = U / R::U4;
    const int u = (U - row * R::U4) ^ ((row >> 2) & 3);
    const int p = p0 + row;
    aoff[j] = (p < a.P ? p : 0) * (kPts * kCh) + 4 * u;  // rows past P read tile 0, never stored
  }
  const bool b_extra = wave < R::B_INS % 4;  // this wave issues NS_HI DMAs per slice
#pragma unroll
  for (int s = 0; s < R::B_PW; ++s) {
    const int q = wave + 4 * s;  // B instruction; >= B_INS: none for this wave
    const int U = (q < R::B_INS ? q : 0) * 64 + lane;
    const int row = U / R::U4;
    const int u = (U - row * R::U4) ^ ((row >> 2) & 3);
    boff[s] = (n0 + row) * kCh + 4 * u;
    bdst[s] = R::A_FL + q * 256;
  }
  lds_f32* lds3 = (lds_f32*)(lds);  // generic -> LDS address space (C-style cast required)

  auto issue = [&](int it) {
    const int ab = it / KS, kk = (it - ab * KS) * BK;
    const float* va = a.V + ab * kCh + kk;
    const float* ub = a.U + static_cast<size_t>(ab) * a.K * kCh + kk;
    lds_f32* st = lds3 + (it % NST) * R::STAGE;
#pragma unroll
    for (int j = 0; j < R::A_PW; ++j) glds16(va + aoff[j], st + (j * 4 + wave) * 256);
#pragma unroll
    for (int s = 0; s < R::B_PW; ++s)
      if (wave + 4 * s < R::B_INS) glds16(ub + boff[s], st + bdst[s]);
  };

  const int r = lane & 31, h = lane >> 5;
  const int swz = (r >> 2) & 3;  // rows wave*32 + r (A) and r (B) share it
  int rd[BK / 8];                // unit (h*BK/8 + s4) of my row, swizzled, in floats
#pragma unroll
  for (int s4 = 0; s4 < BK / 8; ++s4) rd[s4] = 4 * ((h * (BK / 8) + s4) ^ swz);
  const int a_row = (wave * 32 + r) * BK, b_row = R::A_FL + r * BK;

  // Y[q][e2]: output q of accumulator rows 2*e2 and 2*e2+1 (pairs: one v_pk_fma_f32 per 2 rows)
  f32x2 Y[9][8];
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) Y[q][e2] = f32x2{0.f, 0.f};
  f32x16 acc0 = {}, acc1 = {};

  // k permutation inside a slice: lane half h at MFMA step s consumes k = h*BK/2 + s (A and B
  // alike, so the sum is unchanged); one ds_read_b128 per operand feeds 4 MFMAs.
  auto mfma_slice = [&](int it, f32x16& acc) {
    const float* base = lds + (it % NST) * R::STAGE;
#pragma unroll
    for (int s4 = 0; s4 < BK / 8; ++s4) {
      const f32x4 af = *reinterpret_cast<const f32x4*>(base + a_row + rd[s4]);
      const f32x4 bf = *reinterpret_cast<const f32x4*>(base + b_row + rd[s4]);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
    }
  };
  // Y += A^T[i][a] A^T[j][b] M_ab. The coefficients are wave-uniform (scalar registers): a zero one
  // (104 of the 225 coefficient x point pairs) skips its 16 FMAs with a scalar branch.
  auto fold = [&](int ab, f32x16& acc) {
    if (a.probe & 1) {
      acc = f32x16{};
      return;
    }
    const int aa = ab / kN5, bb = ab - aa * kN5;
#pragma unroll
    for (int i3 = 0; i3 < 3; ++i3)
#pragma unroll
      for (int j3 = 0; j3 < 3; ++j3) {
        const float c = c_at33.v[i3][aa] * c_at33.v[j3][bb];
        if (c != 0.f) {
#pragma unroll
          for (int e2 = 0; e2 < 8; ++e2) fma2<SF>(Y[i3 * 3 + j3][e2], c, acc[2 * e2], acc[2 * e2 + 1]);
        }
      }
    acc = f32x16{};
  };
  // one slice: retire slice it (counted wait: the slices issued after it stay in flight), one raw
  // barrier (every wave's DMA of slice it landed; every wave is done reading the slot refilled next)
  auto step = [&](int it, f32x16& acc) {
    const int ahead = TOTAL - 1 - it;  // capped at NST - 2 by wait_ahead
    if (b_extra)
      wait_ahead<R::NS_HI, NST - 2>(ahead);
    else
      wait_ahead<R::NS_LO, NST - 2>(ahead);
    if ((a.probe & 6) != 6) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // keep the DMA refill and the ds_reads below the barrier
    if (it + NST - 1 < TOTAL && !(a.probe & 2)) issue(it + NST - 1);
    if (a.probe & 16) __builtin_amdgcn_s_setprio(1);
    mfma_slice(it, acc);
    if (a.probe & 16) __builtin_amdgcn_s_setprio(0);
  };

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < TOTAL) issue(s);
  // Even points accumulate in acc0, odd in acc1; the fold of point ab-1 is issued after the first
  // slice of point ab, so its VALU work overlaps the in-flight MFMAs.
  int it = 0;
  for (int ab = 0; ab < kPts; ab += 2) {
    for (int ks = 0; ks < KS; ++ks, ++it) {
      step(it, acc0);
      if (ks == 0 && ab > 0) fold(ab - 1, acc1);
    }
    if (ab + 1 < kPts) {
      for (int ks = 0; ks < KS; ++ks, ++it) {
        step(it, acc1);
        if (ks == 0) fold(ab, acc0);
      }
    }
  }
  fold(kPts - 1, acc0);  // kPts is odd: the last point (24, even) is still in acc0

  // Epilogue: bias + ReLU, then one LDS transpose per output position q so each lane stores whole
  // 16-B filter groups: 4 global_store_dwordx4 per lane per q instead of 16 single-dword stores
  // (the dword form was store-issue-bound: a quarter of the kernel at 300 images).
  // D layout: lane (r, h) holds filter n0 + r of wave tiles (e&3) + 8*(e>>2) + 4h.
  __syncthreads();  // the ring is idle (last slice waited with vmcnt(0)); reuse it as scratch
  constexpr int kTS = kBN + 4;                // 36-float rows: 16-B aligned, few bank conflicts
  float* tr = lds + wave * 32 * kTS;          // wave-private 32 tiles x 32 filters
  const float bv = a.bias ? a.bias[n0 + r] : 0.f;
  const OutView o = a.out;
  // the 4 (tile, 4-filter group) pieces this lane stores: piece k = k*64 + lane
  int oy0[4], ox0[4], img[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + wave * 32 + ((k * 64 + lane) >> 3);
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = (p < a.P && !(a.probe & 8)) ? (pq % a.ty) * 3 : (1 << 28);  // out of range: never stored
    ox0[k] = tj * 3;
    img[k] = pq / a.ty;
  }
  const int grp = 4 * (lane & 7);
#pragma unroll
  for (int q = 0; q < 9; ++q) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float v = Y[q][e >> 1][e & 1] + bv;
      if (a.relu) v = fmaxf(v, 0.f);
      tr[((e & 3) + 8 * (e >> 2) + 4 * h) * kTS + r] = v;
    }
    // same-wave LDS accesses complete in order: the reads below see this wave's writes, and the
    // next q's writes cannot overtake these reads
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) >> 3) * kTS + grp);
      const int oy = oy0[k] + q / 3, ox = ox0[k] + q % 3;
      if (oy < a.H1 && ox < a.W1)
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(img[k] * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) *
                                               o.Cb + o.c_off + n0 + grp) = v4;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// The same GEMM on v_mfma_f32_16x16x4_f32 for occupancy. A 32x32 wave tile needs 9 x 16 fold
// registers (Y) and caps the kernel at 2 waves/SIMD; a 16-tile x 32-filter wave tile (two 16x16
// blocks) needs 9 x 8, so 4 workgroups (16 waves) fit a CU. Workgroup = 64 tiles x 32 filters
// (4 waves along the tiles), BK = 48 (one slice per point), 2 ring slots of 18 KiB.
// 16x16x4 operands: lane l holds A[tile l&15][k] and B[k][filter l&15] for the k of lane group
// g = l>>4; lane group g at MFMA step t (0..11) supplies k = 12g + t, so one ds_read_b128 per
// operand feeds 4 steps. D: filter l&15, tile 4g + reg. The LDS image rotates the 16-B units of
// row r by 3*((r>>1)&3) (mod 12): conflict-free for this read pattern (exhaustive check over the
// four ds_read_b128 lane groups), applied on the DMA's global source address.
constexpr int kBM16 = 64;
__device__ __forceinline__ int rot16(int row) { return 3 * ((row >> 1) & 3); }

template <bool IL, bool SF>
__global__ void __launch_bounds__(256, 3) conv1_wino_gemm16_kernel(GemmArgs a) {  // 3 per CU (Knobs::conv1_occ default): 168 VGPRs, no spills
  constexpr int BK = kCh, U4 = BK / 4;            // 48 channels, 12 units per row
  constexpr int A_PW = kBM16 * U4 / 64 / 4;       // 3 DMA instructions per wave
  constexpr int B_INS = kBN * U4 / 64;            // 6
  constexpr int A_FL = kBM16 * BK, B_FL = kBN * BK;
  constexpr int STAGE = A_FL + B_FL;
  constexpr int NS_LO = A_PW + B_INS / 4, NS_HI = NS_LO + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles;
  const int pt = (jb / a.n_ntiles) * 8 + xcd;
  if (pt >= a.n_ptiles) return;  // whole workgroup: before any DMA or barrier
  const int p0 = pt * kBM16, n0 = nt * kBN;

  int aoff[A_PW], boff[2];
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    const int U = (j * 4 + wave) * 64 + lane;
    const int row = U / U4, su = U - row * U4;
    const int u = (su + U4 - rot16(row)) % U4;  // logical unit stored at slot su
    const int p = p0 + row;
    aoff[j] = (p < a.P ? p : 0) * (kPts * kCh) + 4 * u;
  }
  const bool b_extra = wave < B_INS % 4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int q = wave + 4 * s;
    const int U = (q < B_INS ? q : 0) * 64 + lane;
    const int row = U / U4, su = U - row * U4;
    boff[s] = (n0 + row) * kCh + 4 * ((su + U4 - rot16(row)) % U4);
  }
  lds_f32* lds3 = (lds_f32*)(lds);
  // buffer_load ... lds when V fits 31-bit byte offsets (a.vbytes > 0): per-lane offsets in VGPRs once,
  // the per-point offset scalar (no 64-bit VALU address per DMA)
#if __HIP_DEVICE_COMPILE__  // the buffer-resource type exists in the device pass only
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.V), 0, a.vbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
#endif
  auto issue = [&](int ab) {
    lds_f32* st = lds3 + (ab & 1) * STAGE;
#if __HIP_DEVICE_COMPILE__
    if (a.vbytes > 0) {
#pragma unroll
      for (int j = 0; j < A_PW; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (lds_void*)(st + (j * 4 + wave) * 256), 16, aoff[j] * 4,
                                                 ab * kCh * 4, 0, 0);
#pragma unroll
      for (int s = 0; s < 2; ++s)
        if (wave + 4 * s < B_INS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)(st + A_FL + (wave + 4 * s) * 256), 16, boff[s] * 4,
                                                   ab * a.K * kCh * 4, 0, 0);
      return;
    }
#endif
    const float* va = a.V + ab * kCh;
    const float* ub = a.U + static_cast<size_t>(ab) * a.K * kCh;
#pragma unroll
    for (int j = 0; j < A_PW; ++j) glds16(va + aoff[j], st + (j * 4 + wave) * 256);
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (wave + 4 * s < B_INS) glds16(ub + boff[s], st + A_FL + (wave + 4 * s) * 256);
  };

  const int r16 = lane & 15, g = lane >> 4;
  const int a_row = (wave * 16 + r16) * BK, b_row0 = A_FL + r16 * BK, b_row1 = A_FL + (16 + r16) * BK;
  // slot (in floats) of logical unit 3g + s4 in rows of either rotation (A rows wave*16 + r16 and
  // B rows r16, 16 + r16 share (row >> 1) & 3)
  int rd[3];
#pragma unroll
  for (int s4 = 0; s4 < 3; ++s4) rd[s4] = 4 * ((3 * g + s4 + rot16(r16)) % U4);

  f32x2 Y[9][2][2];  // [q][block][reg pair]
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int c = 0; c < 2; ++c) Y[q][c][0] = Y[q][c][1] = f32x2{0.f, 0.f};
  f32x4 acc0[2] = {}, acc1[2] = {};

  auto mfma_point = [&](int ab, f32x4 (&acc)[2]) {
    const float* base = lds + (ab & 1) * STAGE;
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
    if (a.probe & 1) {  // cost probe: keep the accumulators live, skip the output-transform FMAs
      Y[0][0][0] += f32x2{acc[0][0] + acc[1][0], acc[0][1] + acc[1][1]};
      acc[0] = acc[1] = f32x4{};
      return;
    }
    const int aa = ab / kN5, bb = ab - aa * kN5;
#pragma unroll
    for (int i3 = 0; i3 < 3; ++i3)
#pragma unroll
      for (int j3 = 0; j3 < 3; ++j3) {
        const float c = c_at33.v[i3][aa] * c_at33.v[j3][bb];
        if (c != 0.f) {
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            fma2<SF>(Y[i3 * 3 + j3][cb][0], c, acc[cb][0], acc[cb][1]);
            fma2<SF>(Y[i3 * 3 + j3][cb][1], c, acc[cb][2], acc[cb][3]);
          }
        }
      }
    acc[0] = acc[1] = f32x4{};
  };
  auto step = [&](int ab, f32x4 (&acc)[2]) {
    wait_vmcnt<0>();  // this wave's DMA of point ab landed (it was issued one point ago)
    if ((a.probe & 6) != 6) __builtin_amdgcn_s_barrier();  // ... and every other wave's (probe 6: skipped)
    asm volatile("" ::: "memory");
    if (ab + 1 < kPts && !(a.probe & 2)) issue(ab + 1);  // probe 2: no refills (operands stale)
    if (a.probe & 16) __builtin_amdgcn_s_setprio(1);
    mfma_point(ab, acc);
    if (a.probe & 16) __builtin_amdgcn_s_setprio(0);
  };
  // IL: the fold of point fab rides inside the MFMAs of the next point, branch-free (zero
  // coefficients included: +0 leaves Y bit-identical), 3 packed FMAs per MFMA pair, so the VALU
  // work issues while the matrix pipe is busy instead of after it.
  auto point_fold = [&](int ab, f32x4 (&acc)[2], int fab, f32x4 (&facc)[2]) {
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ab + 1 < kPts) issue(ab + 1);
    if (a.probe & 16) __builtin_amdgcn_s_setprio(1);
    float cq[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) cq[q] = c_coef33.v[fab][q];
    const float* base = lds + (ab & 1) * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < 3; ++s4) {
      const f32x4 af = *reinterpret_cast<const f32x4*>(base + a_row + rd[s4]);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(base + b_row0 + rd[s4]);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(base + b_row1 + rd[s4]);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], b0[s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], b1[s], acc[1], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int j = (s4 * 4 + s) * 3 + t;  // 0..35 = (q, cb, pair)
          const int q = j >> 2, cb = (j >> 1) & 1, pr = j & 1;
          fma2<SF>(Y[q][cb][pr], cq[q], facc[cb][2 * pr], facc[cb][2 * pr + 1]);
        }
      }
    }
    facc[0] = facc[1] = f32x4{};
    if (a.probe & 16) __builtin_amdgcn_s_setprio(0);
  };
  (void)b_extra;
  (void)NS_HI;

  issue(0);
  if constexpr (IL) {
    // acc1 is zero before point 1: the first fold adds +0 and changes nothing
    for (int ab = 0; ab + 1 < kPts; ab += 2) {
      point_fold(ab, acc0, ab > 0 ? ab - 1 : 0, acc1);
      point_fold(ab + 1, acc1, ab, acc0);
    }
    point_fold(kPts - 1, acc0, kPts - 2, acc1);
  } else {
    for (int ab = 0; ab < kPts; ab += 2) {
      step(ab, acc0);
      if (ab > 0) fold(ab - 1, acc1);
      if (ab + 1 < kPts) {
        step(ab + 1, acc1);
        fold(ab, acc0);
      }
    }
  }
  fold(kPts - 1, acc0);

  // epilogue: per output position q, transpose the wave's 16 tiles x 32 filters through LDS and
  // store 16-B filter groups (2 per lane)
  __syncthreads();
  constexpr int kTS = kBN + 4;
  float* tr = lds + wave * 16 * kTS;
  float bv[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) bv[cb] = a.bias ? a.bias[n0 + cb * 16 + r16] : 0.f;
  const OutView o = a.out;
  int oy0[2], ox0[2], img[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = p0 + wave * 16 + ((k * 64 + lane) >> 3);
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = (p < a.P && !(a.probe & 8)) ? (pq % a.ty) * 3 : (1 << 28);
    ox0[k] = tj * 3;
    img[k] = pq / a.ty;
  }
  const int grp = 4 * (lane & 7);
#pragma unroll
  for (int q = 0; q < 9; ++q) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        float v = Y[q][cb][reg >> 1][reg & 1] + bv[cb];
        if (a.relu) v = fmaxf(v, 0.f);
        tr[(4 * g + reg) * kTS + cb * 16 + r16] = v;
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) >> 3) * kTS + grp);
      const int oy = oy0[k] + q / 3, ox = ox0[k] + q % 3;
      if (oy < a.H1 && ox < a.W1)
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(img[k] * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) *
                                               o.Cb + o.c_off + n0 + grp) = v4;
    }
  }
}

// GEMM configurations (Knobs::conv1_cfg). 0-3: 32x32 MFMA, 128-tile workgroups, 2 per CU, ring of
// BK channels x NST slots (NST-2 slices in flight behind the one being consumed): 0 BK 48 x 2
// (60 KiB), 1 BK 16 x 4 (40 KiB), 2 BK 16 x 6 (60 KiB), 3 BK 16 x 8 (80 KiB). 4 (default): 16x16 MFMA,
// 64-tile workgroups, 4 per CU (conv1_wino_gemm16_kernel; -6 % kernel time at 300 images,
// profiles/r01_ab_conv1_wino_b300.jsonl).
constexpr int kNumCfg = 5;

template <int BK, int NST, bool SF>
hipError_t launch_gemm_t(const GemmArgs& a, hipStream_t s) {
  constexpr size_t lds_bytes = Ring<BK, NST>::kBytes;
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(conv1_wino_gemm_kernel<BK, NST, SF>), hipFuncAttributeMaxDynamicSharedMemorySize,
      lds_bytes);
  if (attr != hipSuccess) return attr;
  const dim3 grid((a.n_ptiles + 7) / 8 * 8 * a.n_ntiles);
  conv1_wino_gemm_kernel<BK, NST, SF><<<grid, 256, lds_bytes, s>>>(a);
  return hipGetLastError();
}
template <int BK, int NST>
hipError_t launch_gemm(const GemmArgs& a, hipStream_t s, bool sf) {
  return sf ? launch_gemm_t<BK, NST, true>(a, s) : launch_gemm_t<BK, NST, false>(a, s);
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

bool conv1_wino_cfg_valid(int cfg) { return cfg >= 0 && cfg < kNumCfg; }

hipError_t conv1_wino(const Conv1WinoPlan& w, const float* x, float* V, const float* U, const float* bias, OutView out,
                      bool relu, hipStream_t s, const Knobs& kn) {
  const int probe = kn.conv1_probe;
  const bool sf = (kn.fold_scalar & 1) != 0;
  if (w.P == 0 || w.H1 <= 0 || w.W1 <= 0) return hipSuccess;
  if (w.K % kBN || static_cast<long>(w.P) * kPts * kCh >= (1L << 31) || static_cast<long>(w.P) * 12 >= (1L << 31) ||
      out.Cb % 4 || out.c_off % 4)  // 16-B epilogue stores
    return hipErrorInvalidValue;
  const int total = w.P * 12;
  long g = (total + kT - 1) / kT;
  if (g > (1 << 20)) g = 1 << 20;
  if (probe & 32)  // A/B: non-temporal V stores
    conv1_wino_in_kernel<true><<<static_cast<unsigned>(g), kT, 0, s>>>(x, V, total, w.Hin, w.W * 3, w.ty, w.tx);
  else
    conv1_wino_in_kernel<false><<<static_cast<unsigned>(g), kT, 0, s>>>(x, V, total, w.Hin, w.W * 3, w.ty, w.tx);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  GemmArgs a{};
  a.V = V;
  a.U = U;
  a.bias = bias;
  a.out = out;
  a.P = w.P;
  a.K = w.K;
  a.H1 = w.H1;
  a.W1 = w.W1;
  a.ty = w.ty;
  a.tx = w.tx;
  a.relu = relu ? 1 : 0;
  a.n_ptiles = (w.P + kBM - 1) / kBM;
  a.n_ntiles = w.K / kBN;
  a.probe = probe;
  switch (kn.conv1_cfg) {
    case 1: return launch_gemm<16, 4>(a, s, sf);
    case 2: return launch_gemm<16, 6>(a, s, sf);
    case 3: return launch_gemm<16, 8>(a, s, sf);
    case 4: {  // 16x16 MFMA, 64-tile workgroups, 4 workgroups per CU
      const size_t lds_bytes = occupancy_lds(2 * (kBM16 + kBN) * kCh * sizeof(float), kn.conv1_occ);
      static const hipError_t attr = [] {
        for (const void* f : {reinterpret_cast<const void*>(conv1_wino_gemm16_kernel<true, true>),
                              reinterpret_cast<const void*>(conv1_wino_gemm16_kernel<true, false>),
                              reinterpret_cast<const void*>(conv1_wino_gemm16_kernel<false, true>),
                              reinterpret_cast<const void*>(conv1_wino_gemm16_kernel<false, false>)}) {
          const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
          if (e != hipSuccess) return e;
        }
        return hipSuccess;
      }();
      if (attr != hipSuccess) return attr;
      GemmArgs b = a;
      b.n_ptiles = (a.P + kBM16 - 1) / kBM16;
      {  // probe bit 7: global_load_lds operands (A/B)
        const long vb = static_cast<long>(w.P) * kPts * kCh * 4, ub = static_cast<long>(conv1_wino_u_floats(w.K)) * 4;
        const bool buf = !(probe & 128) && vb < (1L << 31) && ub < (1L << 31);
        b.vbytes = buf ? static_cast<int>(vb) : 0;
        b.ubytes = buf ? static_cast<int>(ub) : 0;
      }
      const dim3 grid((b.n_ptiles + 7) / 8 * 8 * b.n_ntiles);
      if (probe & 64) {
        if (sf)
          conv1_wino_gemm16_kernel<true, true><<<grid, 256, lds_bytes, s>>>(b);
        else
          conv1_wino_gemm16_kernel<true, false><<<grid, 256, lds_bytes, s>>>(b);
      } else {
        if (sf)
          conv1_wino_gemm16_kernel<false, true><<<grid, 256, lds_bytes, s>>>(b);
        else
          conv1_wino_gemm16_kernel<false, false><<<grid, 256, lds_bytes, s>>>(b);
      }
      return hipGetLastError();
    }
    default: return launch_gemm<48, 2>(a, s, sf);
  }
}

}  // namespace anx::hip
