// Conv1 of the bf16 full AlexNet (extension, BASELINE config 5) as a persistent row-band kernel.
//
// Conv1 runs on the polyphase input (space-to-depth by the stride: 11x11/4 over 3 channels becomes
// 3x3/1 over 48, full_engine.cpp), x' [N][57][57][48] bf16, 96 filters, 55x55 outputs. As an
// implicit GEMM over 96-row tiles (conv_bf16_big.hip, 8067 workgroups of 96 pixels x 96 filters)
// every K tile gathers its A rows from L2 again: 9 taps x 48 channels per pixel, i.e. the image is
// fetched 9 times over (1.3 GB of L2 -> LDS traffic at 256 images), and the layer ran 113 us
// (profiles/r03_full_bf16_kernels_b256.md) against ~46 us for its HBM bytes.
//
// Here one workgroup (4 waves, one per SIMD) walks an image in tiles of four output rows:
//   * the polyphase rows it needs live in a 10-slot LDS ring (slot = row % 10; a row is 57 x 48 bf16
//     = 5472 B, one LDS-DMA copy of 6 pieces); tile t reads rows 4t .. 4t+5 and the DMAs of rows
//     4t+6 .. 4t+9 (tile t+1) fly behind its MFMAs, so each input row crosses HBM once;
//   * all 96 filters' weights stay in LDS for the kernel's lifetime ([96][440] bf16, row stride 880
//     B: the 32 rows of a 32x32x16 operand read hit distinct bank quads);
//   * wave w owns pixels 64w .. 64w+63 of the tile (220 valid of 256) x all 96 filters: per K step
//     (16 of the 432) two pixel fragments and three filter fragments feed six
//     v_mfma_f32_32x32x16_bf16 (filters as the A operand, so each lane ends up holding 4
//     consecutive filters of one pixel: 8-B stores, no LDS transpose). 5 fragment reads per 6 MFMAs
//     keep the LDS at ~40 % of its rate (the 8-wave 32-pixel form read 4 per 3 and ran the MFMA pipe
//     28 % busy with 21 % of LDS cycles in bank conflicts);
//   * a polyphase column's six 16-B channel units are stored in the order k ^ ((column >> 3) & 1)
//     (applied on the DMA's source side), which halves the pixel reads' bank conflicts;
//   * bias (registers) + ReLU + bf16 in the epilogue, straight into the NHWC output, or with pool1
//     fused (one workgroup per image) through LDS into the pooled map.
// Fragments are read two K steps ahead of their MFMAs (registers triple-buffered).
//
// Reference op: convKernel (final_project/v3_cuda_only/src/layers_cuda.cu:20-46); the full-network
// tail is the extension's own.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "anx/bf16_ops.hpp"
#include "anx/hip_sync.hpp"

namespace anx::hip {
namespace {

using bf16 = __bf16;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned;
using u16x8 = __attribute__((ext_vector_type(8))) unsigned short;
using lds_b16 = __attribute__((address_space(3))) bf16;
using lds_void = __attribute__((address_space(3))) void;

constexpr int kP = 57, kCh = 48, kRowB = kP * kCh * 2;  // polyphase rows: 57 x 48 bf16 = 5472 B
constexpr int kHo = 55, kWo = 55, kK = 96, kKd = 432;  // output rows / cols, filters, GEMM K
constexpr int kSlots = 10, kPieces = 6;                 // ring: 10 rows of 6 DMA pieces (6 KiB)
constexpr int kSlotB = kPieces * 1024 + 16;             // + one 16-B unit: a slot change shifts the banks
constexpr int kWRow = 440;                              // weight row stride (bf16): 880 B
constexpr int kWBytes = 83 * 1024;                      // [96][440] bf16 = 84,480 B, padded to whole DMA pieces
constexpr int kRing = kSlots * kSlotB;                  // 49,152 B
constexpr size_t kLds = kRing + kWBytes;                // 146,592 B
constexpr int kPw = 27, kCarryB = kPw * kK * 2;         // pool1: a pooled row's running max, 5184 B
constexpr size_t kLdsPool = kLds + 2 * kCarryB;         // + two carry rows: 157,344 B
constexpr int kRT = 4;                                  // output rows per tile
constexpr int kTilesPerImage = (kHo + kRT - 1) / kRT;   // 14 (the last holds three rows)
constexpr int kNT = 256, kWaves = kNT / 64, kPB = 2;   // waves, 32-pixel blocks per wave
constexpr int kKS = kKd / 16;                           // 27 K steps (3 per tap)
constexpr int kAhead = 2;                               // K steps of fragments in flight
constexpr int kOOB = 0x7ffffff0;
static_assert(kK * kWRow * 2 <= kWBytes && kRowB <= kPieces * 1024 && kRing % 16 == 0, "LDS layout");
// pool1 scratch rows: a pixel's 48 filters (96 B) at a 112-B stride, so the epilogue's 8-B writes of
// 32 consecutive pixels hit 16 bank offsets (2-way) instead of 8 (4-way at 96 B)
constexpr int kPix = 112;
static_assert(kLdsPool <= 160 * 1024 && kWo * kPix <= kSlotB, "pool1: carry rows fit; a 48-filter output row fits a slot");
static_assert(kWaves * kPB * 32 >= kRT * kWo, "a tile's pixels fit the waves' blocks");
static_assert(kRT * kPieces % kWaves == 0, "a tile's row DMAs split evenly over the waves");
[[maybe_unused]] constexpr int kDPW = kRT * kPieces / kWaves;            // row DMAs per wave per tile (6)
constexpr int kSPW = kPB * 12;                          // output stores per wave per tile (24)

struct Args {
  const void* x;      // F32IN: [N][227][227][3] fp32 images; else [N][57][57][48] bf16 polyphase
  const bf16* w;      // [96][440] (K = tap * 48 + channel, zero past 432), kWBytes bytes
  const float* bias;  // [96]
  bf16* out;          // NHWC through the view
  int Hb, Wb, Cb, h_off, w_off, c_off;
  int N, segs;        // segments per image (workgroups sharing one image's tiles)
  int xbytes, obytes;
  int pool;           // pool1 in the epilogue (F32IN, segs == 1): `out` unused, pooled rows to pout
  bf16* pout;
  int pHb, pWb, pCb, ph_off, pw_off, pc_off;
  unsigned long long* dbg;  // ANX_RING_PHASES: per-workgroup phase clocks (wave 0), else null
};

// bf16(relu(acc[4j .. 4j+3] + bias)): the add as two packed f32 adds, then one packed conversion, then
// ReLU as a signed 16-bit max with 0 on the bf16 bits (a negative value, -0 included, has its sign bit
// set) — bit-identical to fmaxf before the conversion, since the rounding is monotonic
using i16x4 = __attribute__((ext_vector_type(4))) short;
using f32x2 = __attribute__((ext_vector_type(2))) float;
__device__ __forceinline__ bf16x4 bias_relu_bf16(const f32x16& acc, int j, f32x4 bv) {
  const f32x2 lo = f32x2{acc[4 * j], acc[4 * j + 1]} + f32x2{bv[0], bv[1]};
  const f32x2 hi = f32x2{acc[4 * j + 2], acc[4 * j + 3]} + f32x2{bv[2], bv[3]};
  const bf16x4 v = __builtin_convertvector((f32x4{lo[0], lo[1], hi[0], hi[1]}), bf16x4);
  return __builtin_bit_cast(bf16x4, __builtin_elementwise_max(__builtin_bit_cast(i16x4, v), i16x4{0, 0, 0, 0}));
}

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

// F32IN: the space-to-depth and bf16 conversion happen here (the image's fp32 rows are loaded to
// registers one tile ahead and written into the ring converted and swizzled), so neither the
// s2d4 kernel nor its 80 MB polyphase copy runs.
static_assert(kWaves == 4, "F32IN: wave w loads the image rows of phase w");
template <bool F32IN>
__global__ void __launch_bounds__(kNT, 1) conv1_bf16_ring_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = blockIdx.x / a.segs, seg = blockIdx.x - n * a.segs;
  const int t0 = seg * kTilesPerImage / a.segs, t1 = (seg + 1) * kTilesPerImage / a.segs;
  if (n >= a.N || t0 >= t1) return;  // whole workgroup, before any barrier
#if __HIP_DEVICE_COMPILE__
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.w), 0, kWBytes, 0x00020000);
#endif
  [[maybe_unused]] lds_b16* lds3 = (lds_b16*)(lds);

  // ---- kRT polyphase rows into their ring slots: pieces kDPW wave .. +kDPW-1 of the group (each
  // wave issues exactly kDPW DMAs per group: the vmcnt values below are compile-time)
  [[maybe_unused]] auto issue_rows = [&](int row0) {  // rows row0 .. row0 + kRT - 1 (zeros past the image)
#if __HIP_DEVICE_COMPILE__
#pragma unroll
    for (int i = 0; i < kDPW; ++i) {
      const int q = wave * kDPW + i, r = row0 + q / kPieces, pc = q % kPieces;  // wave-uniform
      // LDS unit u of the slot holds column u / 6, channel unit (u % 6) ^ ((column >> 3) & 1)
      const int u = pc * 64 + lane, col = u / 6, k = (u - col * 6) ^ ((col >> 3) & 1);
      const int src = r < kP && u < kP * 6 ? ((n * kP + r) * kRowB + col * (kCh * 2) + k * 16) : kOOB;
      lds_b16* dst = lds3 + ((r % kSlots) * kSlotB + pc * 1024) / 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)dst, 16, src, 0, 0, 0);
    }
#endif
  };

  // ---- F32IN: polyphase rows from the fp32 image. A group of kRT polyphase rows is 16 image rows;
  // wave w loads the rows with phase rh = w (one per polyphase row j), lane c = polyphase column c
  // (57 of 64 lanes): 12 floats (4 image columns x 3 channels) -> 12 bf16 at channels 12 rh .. +11
  // of column c, written as three 8-B pieces at their swizzled 16-B units. The 12 floats are three
  // 16-B loads at 4-B alignment (HSA runs buffer accesses in unaligned mode); column 56 has 9 floats
  // and its third load takes the row's last 16 B (floats 5..8), so no load reaches past the tensor.
  [[maybe_unused]] f32x4 xw[kRT][3];
  [[maybe_unused]] auto row_of = [&](int row0, int jj, int& row, bool& ok) {
    const int pr = row0 + jj;
    row = 4 * pr + wave;
    ok = pr < kP && row < 227;
  };
  [[maybe_unused]] auto load_units = [&](int row0) {  // polyphase rows row0 .. row0 + kRT - 1 into xw
#if __HIP_DEVICE_COMPILE__
    const int c = lane;
#pragma unroll
    for (int jj = 0; jj < kRT; ++jj) {
      int row;
      bool ok;
      row_of(row0, jj, row, ok);
      const int b = ok && c < kP ? ((n * 227 + row) * 681 + 12 * c) * 4 : kOOB;
      xw[jj][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, b, 0, 0));
      xw[jj][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, b, 16, 0));
      xw[jj][2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, b + (c == kP - 1 ? 20 : 32), 0, 0));
    }
#endif
  };
  [[maybe_unused]] auto store_units = [&](int row0) {
    const int c = lane, sw = (c >> 3) & 1;
    if (c >= kP) return;
#pragma unroll
    for (int jj = 0; jj < kRT; ++jj) {
      int row;
      bool ok;
      row_of(row0, jj, row, ok);
      float u[12];
#pragma unroll
      for (int f = 0; f < 12; ++f) u[f] = xw[jj][f >> 2][f & 3];
      u[8] = c == kP - 1 ? xw[jj][2][3] : u[8];
#pragma unroll
      for (int f = 0; f < 12; ++f) u[f] = ok && !(c == kP - 1 && f >= 9) ? u[f] : 0.f;  // column 227 / past the image
      char* col = lds + ((row0 + jj) % kSlots) * kSlotB + c * (kCh * 2);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int lb = wave * 24 + q * 8;  // logical byte in the column's 96 (rh = wave)
        // one packed conversion per pair (element-wise casts became a cvt with a zero partner + a perm)
        const bf16x4 v = __builtin_convertvector((f32x4{u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]}), bf16x4);
        *reinterpret_cast<bf16x4*>(col + (((lb >> 4) ^ sw) << 4) + (lb & 15)) = v;
      }
    }
  };

  // ---- prologue: weights + bias, the first tile's 6 rows (two groups)
#if __HIP_DEVICE_COMPILE__
  for (int q = wave; q < kWBytes / 1024; q += kWaves)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void*)(lds3 + (kRing + q * 1024) / 2), 16, q * 1024 + lane * 16, 0,
                                             0, 0);
#endif
  if constexpr (F32IN) {
    load_units(kRT * t0);
    store_units(kRT * t0);
    load_units(kRT * t0 + kRT);
    store_units(kRT * t0 + kRT);
  } else {
    issue_rows(kRT * t0);
    issue_rows(kRT * t0 + kRT);
  }

  // ---- per-lane fragment addressing. Pixel operand: lane (r, h) reads pixel m = 64 wave + 32 b + r,
  // channels 16 c + 8 h .. +7 of tap (qh, qw) (unit 2c + h, swizzled); filter operand: filter
  // 32 nb + r, K 16 ks + 8 h .. +7.
  const int r = lane & 31, h = lane >> 5;
  int mrow[kPB], ox[kPB], po[kPB][3];
#pragma unroll
  for (int b = 0; b < kPB; ++b) {
    const int m = 64 * wave + 32 * b + r;
    mrow[b] = m < kRT * kWo ? m / kWo : 0;
    ox[b] = m < kRT * kWo ? m - mrow[b] * kWo : 0;
#pragma unroll
    for (int qw = 0; qw < 3; ++qw) {
      const int c = ox[b] + qw;
      po[b][qw] = c * (kCh * 2) + (h ^ ((c >> 3) & 1)) * 16;
    }
  }
  const int wbase = kRing + r * (kWRow * 2) + h * 16;
  f32x16 acc[kPB][3];
  bf16x8 pf[kAhead + 1][kPB], wf[kAhead + 1][3];

#if __HIP_DEVICE_COMPILE__
  const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.obytes, 0x00020000);
#endif
  // the lane's 48 bias values (filters 32 nb + 8 j + 4 h + 0..3) in registers for the kernel's
  // lifetime: read from LDS per 4-filter group, each read's wait serialised the epilogue on LDS latency
  f32x4 bias_r[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) bias_r[q] = *reinterpret_cast<const f32x4*>(a.bias + 32 * (q / 4) + 8 * (q % 4) + 4 * h);
  // consume them here: the compiler's wait for these loads otherwise lands in every tile's epilogue
  // as vmcnt waits that also wait for the next tile's row loads issued before it
#pragma unroll
  for (int q = 0; q < 12; ++q) asm volatile("" : "+v"(bias_r[q]));
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tc = __builtin_amdgcn_s_memtime();
  auto lap = [&](int i) {
    if (a.dbg) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      ph[i] += now - tc;
      tc = now;
    }
  };
  for (int t = t0; t < t1; ++t) {
    // Rows 4t .. 4t+5 landed: this wave's DMAs by a counted vmcnt (vmcnt is in order; the last group,
    // rows 4t+2 .. 4t+5, was issued at tile t-1's start and only tile t-1's kSPW output stores per
    // wave followed it; the first tile waits for the prologue), every wave's by the barrier, which
    // also retires tile t-1's reads of the slots refilled below.
    if (t == t0)
      lds_barrier<0>();
    else if constexpr (F32IN)  // the rows were written by ds_write at tile t-1's end
      lds_barrier<>();
    else
      lds_barrier<kSPW>();
    asm volatile("" ::: "memory");
    lap(0);
    if (t + 1 < t1) {  // tile t+1's new rows, into tile t-1's first slots
      if constexpr (F32IN)
        load_units(kRT * t + 6);
      else
        issue_rows(kRT * t + 6);
    }
    int sb[kPB][3];
#pragma unroll
    for (int b = 0; b < kPB; ++b)
#pragma unroll
      for (int qh = 0; qh < 3; ++qh) sb[b][qh] = ((kRT * t + mrow[b] + qh) % kSlots) * kSlotB;
    auto pix = [&](int ks, int b) -> bf16x8 {  // ks compile-time after unrolling
      const int tap = ks / 3, qh = tap / 3, qw = tap - 3 * qh, c16 = ks - 3 * tap;
      return *reinterpret_cast<const bf16x8*>(lds + sb[b][qh] + po[b][qw] + c16 * 32);
    };
    auto wgt = [&](int ks, int nb) -> bf16x8 {
      return *reinterpret_cast<const bf16x8*>(lds + wbase + nb * 32 * (kWRow * 2) + ks * 32);
    };
    auto load_step = [&](int ks, int set) {
#pragma unroll
      for (int b = 0; b < kPB; ++b) pf[set][b] = pix(ks, b);
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) wf[set][nb] = wgt(ks, nb);
    };
#pragma unroll
    for (int b = 0; b < kPB; ++b)
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) acc[b][nb] = f32x16{};
    // fragments kAhead K steps ahead, each step's reads pinned above the previous step's MFMAs
    // (left alone, the compiler re-read right before each MFMA and waited on it)
    sfor<0, kAhead>([&](auto KS) { load_step(decltype(KS)::value, decltype(KS)::value); });
    sfor<0, kKS>([&](auto KS) {
      constexpr int ks = decltype(KS)::value, cur = ks % (kAhead + 1), nxt = (ks + kAhead) % (kAhead + 1);
      constexpr int per = kPB + 3;  // fragment reads per step
      if constexpr (ks + kAhead < kKS) load_step(ks + kAhead, nxt);
      // this step's fragments landed (the reads of the steps ahead may fly)
      if constexpr (ks + kAhead < kKS)
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(per * kAhead) : "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(per * (kKS - 1 - ks)) : "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b = 0; b < kPB; ++b)
#pragma unroll
        for (int nb = 0; nb < 3; ++nb)
          acc[b][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[cur][nb], pf[cur][b], acc[b][nb], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });

    lap(1);
    // ---- pool1 epilogue (one workgroup per image, tiles in order): the tile's ReLU'd rows go to
    // LDS as bf16, 48 filters at a time, into the ring slots of polyphase rows 4t .. 4t+3 (no wave
    // reads those again: tile t+1 reads rows 4t+4 .. 4t+9, and this tile's store_units fills the
    // slots of rows 4t-4 .. 4t-1). Pooled row 2t is rows 4t .. 4t+2; row 2t-1 is the carried max of
    // rows 4t-2, 4t-1 with row 4t; rows 4t+2, 4t+3 are carried for row 2t+1. Max over ReLU outputs
    // (>= 0) is the unsigned max of their bf16 bits.
    if (F32IN && a.pool) {
      lds_barrier<>();  // every wave is past its fragment reads of the scratch slots
      asm volatile("" ::: "memory");
      lap(4);
      const char* carry_old = lds + kLds + ((t & 1) ^ 1) * kCarryB;
      char* carry_new = lds + kLds + (t & 1) * kCarryB;
      sfor<0, 2>([&](auto P) {
        constexpr int p = decltype(P)::value;
#pragma unroll
        for (int b = 0; b < kPB; ++b) {
          const int m = 64 * wave + 32 * b + r, oy = kRT * t + mrow[b];
          if (m < kRT * kWo && oy < kHo) {
            char* px = lds + ((kRT * t + mrow[b]) % kSlots) * kSlotB + ox[b] * kPix;
            sfor<0, 12>([&](auto Q) {
              constexpr int nb = decltype(Q)::value / 4, j = decltype(Q)::value % 4, f0 = 32 * nb + 8 * j;
              if constexpr (f0 >= 48 * p && f0 < 48 * p + 48) {
                const f32x4 bv = bias_r[nb * 4 + j];
                const bf16x4 v = bias_relu_bf16(acc[b][nb], j, bv);
                *reinterpret_cast<bf16x4*>(px + (f0 - 48 * p + 4 * h) * 2) = v;
              }
            });
          }
        }
        lap(5);
        lds_barrier<>();  // this wave's rows written before the barrier
        asm volatile("" ::: "memory");
        lap(6);
        if (tid < kPw * 6) {  // (pooled column, 8-filter chunk of this half)
          const int pc = tid / 6, c = tid - pc * 6;
          const int cofs = pc * (kK * 2) + (48 * p + 8 * c) * 2;
          // all 13 reads first, one wait (row 3 of the last tile and the carry at the first tile are
          // read but unused)
          u16x8 v[kRT][3];
#pragma unroll
          for (int k = 0; k < kRT; ++k) {
            const char* q = lds + ((kRT * t + k) % kSlots) * kSlotB + 2 * pc * kPix + c * 16;
#pragma unroll
            for (int d = 0; d < 3; ++d) v[k][d] = *reinterpret_cast<const u16x8*>(q + d * kPix);
          }
          const u16x8 co = *reinterpret_cast<const u16x8*>(carry_old + cofs);
          u16x8 hr[kRT];
#pragma unroll
          for (int k = 0; k < kRT; ++k) hr[k] = __builtin_elementwise_max(__builtin_elementwise_max(v[k][0], v[k][1]), v[k][2]);
          const int ob = ((n * a.pHb + a.ph_off) * a.pWb + pc + a.pw_off) * a.pCb + a.pc_off + 48 * p + 8 * c;
          const int rstride = a.pWb * a.pCb;
          *reinterpret_cast<u16x8*>(a.pout + ob + 2 * t * rstride) =
              __builtin_elementwise_max(__builtin_elementwise_max(hr[0], hr[1]), hr[2]);
          if (t > t0)
            *reinterpret_cast<u16x8*>(a.pout + ob + (2 * t - 1) * rstride) = __builtin_elementwise_max(co, hr[0]);
          if (t + 1 < t1) *reinterpret_cast<u16x8*>(carry_new + cofs) = __builtin_elementwise_max(hr[2], hr[3]);
        }
        lap(7);
        if constexpr (p == 0) {
          lds_barrier<>();  // the second half overwrites the scratch rows
          asm volatile("" ::: "memory");
        }
      });
    } else {
      // ---- epilogue: lane holds pixel m, filters 32 nb + 8 j + 4 h + (0..3) in acc[b][nb][4 j .. 4 j + 3].
      // kSPW buffer stores per lane, always issued (a pixel outside the tile stores past the extent,
      // which drops the write), so the vmcnt counts above hold on every wave.
#pragma unroll
      for (int b = 0; b < kPB; ++b) {
        const int m = 64 * wave + 32 * b + r, oy = kRT * t + mrow[b];
        const bool ok = m < kRT * kWo && oy < kHo;
        // the lane's filter half (4 h) rides in the VGPR offset: the SGPR offset must be wave-uniform,
        // or the compiler runs each store as a two-pass waterfall loop (twice the store instructions,
        // which also broke the vmcnt counts above)
        [[maybe_unused]] const int obase =
            ok ? (((n * a.Hb + oy + a.h_off) * a.Wb + ox[b] + a.w_off) * a.Cb + a.c_off + 4 * h) * 2 : kOOB;
#pragma unroll
        for (int nb = 0; nb < 3; ++nb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            [[maybe_unused]] const int f0 = 32 * nb + 8 * j;  // wave-uniform
            const f32x4 bv = bias_r[nb * 4 + j];
            [[maybe_unused]] const bf16x4 v = bias_relu_bf16(acc[b][nb], j, bv);
#if __HIP_DEVICE_COMPILE__
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), orr, obase, f0 * 2, 0);
#endif
          }
      }
    }
    // F32IN: tile t+1's new rows (loaded at this tile's start) into tile t-1's slots, which no wave
    // reads in tile t; the next tile's barrier publishes them
    lap(2);
    if constexpr (F32IN)
      if (t + 1 < t1) store_units(kRT * t + 6);
    lap(3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  if (a.dbg && tid == 0 && blockIdx.x < 64)
    for (int i = 0; i < 8; ++i) a.dbg[blockIdx.x * 8 + i] = ph[i];
}

}  // namespace

void pack_conv1_ring_weights(const float* w_k48_33, std::vector<uint16_t>& out) {
  out.assign(kWBytes / 2, 0);
  for (int k = 0; k < kK; ++k)
    for (int c = 0; c < kCh; ++c)
      for (int qh = 0; qh < 3; ++qh)
        for (int qw = 0; qw < 3; ++qw)
          out[static_cast<size_t>(k) * kWRow + (qh * 3 + qw) * kCh + c] =
              f32_to_bf16_bits(w_k48_33[((static_cast<size_t>(k) * kCh + c) * 3 + qh) * 3 + qw]);
}

size_t conv1_ring_weight_bytes() { return kWBytes; }

hipError_t conv1_bf16_ring(const void* xin, int N, const void* wpacked, const float* bias, OutViewB out, bool relu,
                           hipStream_t s, int cus, bool f32_input, const OutViewB* pool_out) {
  if (N <= 0) return hipSuccess;
  if (!relu || !out.base || out.Cb % 4 || out.c_off % 4 || static_cast<long>(N) * kP * kRowB >= (1L << 31) ||
      static_cast<long>(N) * out.Hb * out.Wb * out.Cb * 2 >= (1L << 31) || out.Hb < kHo + out.h_off ||
      out.Wb < kWo + out.w_off || out.Cb < kK + out.c_off)
    return hipErrorInvalidValue;
  static const hipError_t attr = [] {
    for (const void* k : {reinterpret_cast<const void*>(conv1_bf16_ring_kernel<false>),
                          reinterpret_cast<const void*>(conv1_bf16_ring_kernel<true>)}) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }();
  if (attr != hipSuccess) return attr;
  Args a{};
  a.x = xin;
  if (f32_input && (reinterpret_cast<uintptr_t>(xin) & 3)) return hipErrorInvalidValue;
  a.w = static_cast<const bf16*>(wpacked);
  a.bias = bias;
  a.out = out.base;
  a.Hb = out.Hb;
  a.Wb = out.Wb;
  a.Cb = out.Cb;
  a.h_off = out.h_off;
  a.w_off = out.w_off;
  a.c_off = out.c_off;
  a.N = N;
  // one image per workgroup when the batch fills the CUs; else each image's 14 tiles split over
  // segments (each re-stages its first rows)
  a.segs = std::max(1, std::min(kTilesPerImage / 2, (std::max(1, cus) + N - 1) / N));
  const long xb = f32_input ? static_cast<long>(N) * 227 * 227 * 3 * 4 : static_cast<long>(N) * kP * kRowB;
  if (xb >= (1L << 31)) return hipErrorInvalidValue;
  a.xbytes = static_cast<int>(xb);
  a.obytes = static_cast<int>(static_cast<long>(N) * out.Hb * out.Wb * out.Cb * 2);
  if (pool_out) {
    const OutViewB& q = *pool_out;
    if (!q.base || q.Cb % 8 || q.c_off % 8 || q.Hb < kPw + q.h_off || q.Wb < kPw + q.w_off || q.Cb < kK + q.c_off ||
        static_cast<long>(N) * q.Hb * q.Wb * q.Cb >= (1L << 31))
      return hipErrorInvalidValue;
    a.pool = f32_input && a.segs == 1;
    a.pout = q.base;
    a.pHb = q.Hb;
    a.pWb = q.Wb;
    a.pCb = q.Cb;
    a.ph_off = q.h_off;
    a.pw_off = q.w_off;
    a.pc_off = q.c_off;
    if (!a.pool && (out.Hb != kHo || out.Wb != kWo || out.Cb != kK || out.h_off || out.w_off || out.c_off))
      return hipErrorInvalidValue;  // the separate pool below reads a dense 55x55x96 map
  }
  static const bool phases = std::getenv("ANX_RING_PHASES") != nullptr;
  if (phases) {
    static unsigned long long* dbg = nullptr;
    if (!dbg && hipMalloc(&dbg, 64 * 8 * 8) != hipSuccess) return hipErrorOutOfMemory;
    a.dbg = dbg;
  }
  if (f32_input)
    conv1_bf16_ring_kernel<true><<<static_cast<unsigned>(N * a.segs), kNT, a.pool ? kLdsPool : kLds, s>>>(a);
  else
    conv1_bf16_ring_kernel<false><<<static_cast<unsigned>(N * a.segs), kNT, kLds, s>>>(a);
  if (phases) {  // debug: per-phase s_memtime clocks summed over the tiles, workgroups 0..63 averaged
    unsigned long long h[64 * 8];
    if (hipStreamSynchronize(s) == hipSuccess && hipMemcpy(h, a.dbg, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
      double m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      const int nb = std::min(64, N * a.segs);
      for (int b = 0; b < nb; ++b)
        for (int i = 0; i < 8; ++i) m[i] += static_cast<double>(h[b * 8 + i]) / nb;
      std::fprintf(stderr,
                   "ring phases (clk/workgroup): barrier-wait %.0f  loads+mfma %.0f  epilogue %.0f  store_units %.0f"
                   "  | pool1: drain+barrier %.0f  lds-write %.0f  barrier %.0f  pool %.0f\n",
                   m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]);
    }
  }
  if (pool_out && !a.pool) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return maxpool_bf16(out.base, N, kHo, kWo, kK, 3, 2, *pool_out, s);
  }
  return hipGetLastError();
}

}  // namespace anx::hip
