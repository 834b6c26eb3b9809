// Wide-tile bf16 implicit-GEMM convolution for the full-AlexNet extension (conv1-polyphase, conv2-5).
//
// The 128x128 4-wave kernels of conv_bf16.hip run 2-3 workgroups per CU and measured 0.55-0.70
// PFLOP/s on conv2-5 (profiles/r01_full_bf16_glds_kernels_latest.md): the 128^2 structure's ceiling
// (cdna_hip_programming.md §5, "the step-3 structure"). This kernel is the 1-workgroup-per-CU
// shape: a BM=256-row output tile over 8 waves, operands staged global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, per-lane gather addresses: A row = the output pixel's input-window
// origin + koff of the K slice's tap, B row = packed filter row) into two K=64 buffers, a counted
// vmcnt and one raw barrier per K tile, 16x16x32 bf16 MFMAs in between (setprio-fenced clusters).
//
//   LDS image: rows of 64 bf16 = 8 16-B chunks; chunk c of row r is stored at c ^ ((r >> 1) & 7)
//   (the swizzle lives on the DMA SOURCE address — the DMA destination is lane-linear — and on the
//   fragment reads), so every ds_read_b128 lane group of a 16x16x32 fragment hits 16 distinct bank
//   quads.
//   Tile order: blockIdx -> tile is XCD-aware and bijective (each XCD walks a contiguous run of
//   M tiles: neighbouring output rows share input rows in its L2).
//   Epilogue: bias + ReLU + bf16 into an LDS image of the whole output tile (chunk-XOR swizzled),
//   then 16-B row-contiguous stores — the MFMA C layout (one column per lane) would otherwise
//   store 2 bytes per lane.
//
// Conv reference: final_project/v3_cuda_only/src/layers_cuda.cu:20-62 (one thread per output,
// fp32); the AlexNet tail (conv3-5) is the extension's own (BASELINE.json config 5).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "anx/bf16_ops.hpp"
#include "anx/hip_sync.hpp"

namespace anx::hip {
namespace {

using bf16 = __bf16;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
using lds_b16 = __attribute__((address_space(3))) bf16;

constexpr int kBK = 64;  // bf16 per staged row = 8 chunks of 16 B

struct ArgsW {
  const bf16* x;
  const bf16* w;
  const int* koff;
  const float* bias;
  bf16* out;
  int M, HoWo, Wo, Hp, Wp, C, S, F, Cg, Kg, kpad, kpad_n, ktiles, n_ntiles, m_tiles;
  int Hb, Wb, Cb, h_off, w_off, c_off, relu;
  int kt_per;  // K tiles per blockIdx.y slice (split-K; = ktiles when not split)
  float* ws;   // split-K: fp32 partial slabs [gridDim.y][M][Kg] (no bias / ReLU)
};

__device__ __forceinline__ void glds16(const bf16* g, lds_b16* l) { __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// BM x BN output tile, WGM x WGN waves (WM = BM/WGM rows, WN = BN/WGN columns per wave), NST LDS
// stages (NST - 1 K tiles in flight behind the one being multiplied). SLAB: split-K partial (K tiles
// [y*kt_per, (y+1)*kt_per) of slice y = blockIdx.y) stored as fp32 straight from the accumulators
// into slab y (groups == 1; the reduce adds bias and ReLU).
// PIPE: both k-steps' fragments are read up front (k-step 1's behind the next tile's DMA issue) and
// the 2 x TM x TN MFMAs run on registers already loaded (sched_barrier-fenced), instead of the
// compiler's read-2-wait-8-MFMA interleave that stalls both waves of a SIMD on LDS latency together.
template <int BM, int BN, int WGM, int WGN, int NST, bool SLAB, bool PIPE = false>
__global__ void __launch_bounds__(64 * WGM * WGN) conv_bf16_big_kernel(ArgsW a) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && BM % 16 == 0, "tile split");
  constexpr int UNITS = (BM + BN) * 8;              // 16-B DMA units per stage (A rows, then B rows)
  constexpr int NJ = (UNITS + NT - 1) / NT;         // DMA instructions per lane per stage
  static_assert(UNITS % 64 == 0, "a DMA instruction never straddles A and B");
  constexpr int STAGE = (BM + BN) * kBK;            // bf16 per stage
  constexpr int CH = BN / 8;                        // 16-B chunks per epilogue row
  // epilogue image rows: padded by one 16-B chunk where the image still fits the stages (row r at
  // bank offset 4 * (EW / 8) * r mod 64: 16 consecutive rows on distinct banks), else chunk-XOR
  // swizzled (a 12-chunk row, BN = 96, only permutes within 4 chunks: 4-way conflicts, 23 % of
  // the 128x96 conv1 kernel's LDS cycles)
  constexpr bool EPAD = BM * (BN + 8) <= NST * STAGE;
  constexpr int EW = EPAD ? BN + 8 : BN;
  constexpr int XM = EPAD ? 0 : (CH % 8 == 0) ? 7 : (CH % 4 == 0) ? 3 : (CH % 2 == 0) ? 1 : 0;
  static_assert(BM * EW <= NST * STAGE, "the epilogue image fits in the stages");
  static_assert(NST == 2 || UNITS % NT == 0, "counted vmcnt: every wave issues NJ pieces per stage");
  extern __shared__ __attribute__((aligned(16))) bf16 lds_b[];
  int* ooff_s = reinterpret_cast<int*>(lds_b + NST * STAGE);  // output offset per tile row (-1 past M)

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int wm = wave / WGN, wn = wave % WGN, g = blockIdx.z;
  // XCD-aware bijective remap: dispatch round-robins blocks over the 8 XCDs; give each XCD a
  // contiguous run of tiles (m-major, n inner) so neighbouring tiles share its L2.
  int tile;
  {
    const int nwg = gridDim.x, b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int mt = tile / a.n_ntiles, nt = tile - mt * a.n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const bf16* x = a.x + g * a.Cg;
  const bf16* wg = a.w + static_cast<size_t>(g) * a.kpad_n * a.kpad;
  for (int i = tid; i < BM; i += NT) {
    const int m = m0 + i;
    int oo = -1;
    if (m < a.M) {
      const int n = m / a.HoWo, rr = m - n * a.HoWo, oy = rr / a.Wo, ox = rr - oy * a.Wo;
      oo = ((n * a.Hb + oy + a.h_off) * a.Wb + ox + a.w_off) * a.Cb + a.c_off;
    }
    ooff_s[i] = oo;
  }
  // DMA unit q = j*NT + tid: row q/8 (rows < BM are A rows), physical chunk tid&7 holding logical
  // chunk u (the row-swizzle involution; (row >> 1) & 7 depends on tid only since NT/8 % 16 == 0)
  static_assert((NT / 8) % 16 == 0, "swizzle phase is per-lane");
  const int u = (tid & 7) ^ ((tid >> 4) & 7);
  const bf16* src[NJ];
  bool isA[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int row = j * (NT / 8) + (tid >> 3);
    isA[j] = row < BM;
    if (row < BM) {
      const int m = m0 + row;
      int o = 0;
      if (m < a.M) {
        const int n = m / a.HoWo, rr = m - n * a.HoWo, oy = rr / a.Wo, ox = rr - oy * a.Wo;
        o = ((n * a.Hp + oy * a.S) * a.Wp + ox * a.S) * a.C;
      }
      src[j] = x + o;  // + koff of (K tile, u) per stage
    } else {
      const int n = min(n0 + row - BM, a.kpad_n - 1);  // rows past the packed filters: never stored
      src[j] = wg + static_cast<size_t>(n) * a.kpad + u * 8;  // + kb per stage
    }
  }
  __syncthreads();  // ooff_s visible
  lds_b16* lds3 = (lds_b16*)(lds_b);
  const int kt0 = blockIdx.y * a.kt_per, total = min(a.ktiles - kt0, a.kt_per);
  // This lane's K unit k = kt*64 + 8u as (filter row fh, column fw, channel c): the packer's k order
  // (fh*F + fw)*Cg + c, so its input offset is (fh*Wp + fw)*C + c — the koff table in arithmetic,
  // advanced by one K tile per issue (the issues run in K order). fh == F: K padding (zero-packed
  // weights then meet pixel data at offset 0).
  int uc, ufw, ufh;
  {
    const int k = kt0 * kBK + u * 8, tap = k / a.Cg;
    uc = k - tap * a.Cg;
    ufh = tap / a.F;
    ufw = tap - ufh * a.F;
  }
  auto issue = [&](int kt, int st) {
    const int kb = kt * kBK;
    const int ko = ufh < a.F ? (ufh * a.Wp + ufw) * a.C + uc : 0;
    uc += kBK;
    while (uc >= a.Cg) {
      uc -= a.Cg;
      if (++ufw == a.F) {
        ufw = 0;
        ++ufh;
      }
    }
    lds_b16* dst = lds3 + st * STAGE;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int q0 = j * NT + wave * 64;
      if (UNITS % NT != 0 && q0 >= UNITS) break;  // wave-uniform
      glds16(src[j] + (isA[j] ? ko : kb), dst + q0 * 8);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment reads: lane row (lane & 15) of each 16-row block, k chunk 4s + (lane >> 4); every
  // block starts at a multiple of 16 rows, so the swizzle phase is ((lane & 15) >> 1) & 7
  const int hq = lane >> 4, sw = (lane >> 1) & 7;
  const int arow = (wm * WM + (lane & 15)) * kBK, brow = (BM + wn * WN + (lane & 15)) * kBK;
#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < total) issue(kt0 + i, i);
  int st = 0, st_free = NST - 1;  // stage of tile it; stage of tile it-1 (free once all waves pass)
  for (int it = 0; it < total; ++it) {
    if (it + NST - 2 < total)
      lds_barrier<NJ * (NST - 2)>();  // this lane's pieces of tile it landed (later tiles may fly), every lane's
    else                              // after the barrier; and every wave is done reading tile it-1
      lds_barrier<0>();
    asm volatile("" ::: "memory");
    const bf16* base = lds_b + st * STAGE;
    st = st + 1 == NST ? 0 : st + 1;
    if constexpr (PIPE) {
      bf16x8 a0[TM], b0[TN], a1[TM], b1[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(base + arow + i * 16 * kBK + (hq ^ sw) * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(base + brow + j * 16 * kBK + (hq ^ sw) * 8);
      __builtin_amdgcn_sched_barrier(0);
      if (it + NST - 1 < total) issue(kt0 + it + NST - 1, st_free);
      st_free = st_free + 1 == NST ? 0 : st_free + 1;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a1[i] = *reinterpret_cast<const bf16x8*>(base + arow + i * 16 * kBK + ((4 + hq) ^ sw) * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b1[j] = *reinterpret_cast<const bf16x8*>(base + brow + j * 16 * kBK + ((4 + hq) ^ sw) * 8);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a0[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a1[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      continue;
    }
    if (it + NST - 1 < total) issue(kt0 + it + NST - 1, st_free);
    st_free = st_free + 1 == NST ? 0 : st_free + 1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < kBK / 32; ++s) {
      const int ca = ((4 * s + hq) ^ sw) * 8;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(base + arow + i * 16 * kBK + ca);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(base + brow + j * 16 * kBK + ca);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  // The MFMAs take the filters as the A operand and the pixels as B, so acc[i][j] is the 16x16 tile
  // transposed: lane holds pixel m = ... + (lane & 15), channels n = ... + 4 * (lane >> 4) + e,
  // e = 0..3 — four consecutive channels of one pixel (one 8-B / 16-B write instead of four).
  const int mcol = lane & 15;
  if constexpr (SLAB) {  // 16 pixels x 16 channels per store instruction, 16 B per lane
    float* ws = a.ws + static_cast<size_t>(blockIdx.y) * a.M * a.Kg;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int f = n0 + wn * WN + j * 16 + hq * 4;
      if (f >= a.Kg) continue;  // Kg % 8 == 0: a 4-channel group is wholly in or out
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * WM + i * 16 + mcol;
        if (m < a.M) *reinterpret_cast<f32x4*>(ws + static_cast<size_t>(m) * a.Kg + f) = acc[i][j];
      }
    }
    return;
  }
  // epilogue: the tile through LDS (all DMA retired above; wait for every wave's last reads)
  lds_barrier<>();
  asm volatile("" ::: "memory");
  bf16* E = lds_b;
  using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WN + j * 16 + hq * 4, f = n0 + nl;
    const f32x4 bv = (a.bias && f < a.Kg) ? *reinterpret_cast<const f32x4*>(a.bias + g * a.Kg + f) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * WM + i * 16 + mcol;
      f32x4 v = acc[i][j] + bv;
      if (a.relu) v = f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
      *reinterpret_cast<bf16x4*>(E + ml * EW + (((nl >> 3) ^ (ml & XM)) << 3) + (nl & 7)) =
          bf16x4{static_cast<bf16>(v.x), static_cast<bf16>(v.y), static_cast<bf16>(v.z), static_cast<bf16>(v.w)};
    }
  }
  __syncthreads();
  bf16* out = a.out + g * a.Kg;
  for (int q = tid; q < BM * CH; q += NT) {
    const int ml = q / CH, c = q - ml * CH;
    const int o = ooff_s[ml], f = n0 + c * 8;
    if (o >= 0 && f < a.Kg)
      *reinterpret_cast<u32x4*>(out + o + f) = *reinterpret_cast<const u32x4*>(E + ml * EW + ((c ^ (ml & XM)) << 3));
  }
}

// ---- cfg 12: 256x256 ping-pong (8 waves as two staggered groups) ----
// Group G = wave >> 2 (waves 0-3 / 4-7; wave w runs on SIMD w % 4, so every SIMD holds one wave of
// each group). Group G owns A rows [128 G, 128 G + 128) (its waves are the wm == G row of the 2 x 4
// wave grid) and loads them; each group loads half of the B rows. G1 executes one extra barrier
// first, so one group's fragment reads and DMA issue (L) run while the other group's 64 MFMAs (M)
// own the SIMD's matrix pipe (cdna_hip_programming.md §5, the 8-phase template's stagger).
// LDS: A in 2 stages, B in 3 (5 x 32 KiB = 160 KiB). With #0 the prologue barrier:
//   G0: L_t = (#2t, #2t+1), M_t = (#2t+1, #2t+2);  G1: L_t = (#2t+1, #2t+2), M_t = (#2t+2, #2t+3)
//   G0 in L_t issues A_{t+1} (own rows) and B_{t+1} (rows 0-127) and retires them (vmcnt 0) at the
//   end of M_t; G1 in L_t issues A_{t+1} (own rows) and B_{t+2} (rows 128-255, two tiles ahead:
//   hence 3 B stages), retires B_{t+1} at the end of L_t (vmcnt 8) and A_{t+1} at the end of M_t
//   (vmcnt 4). Every L section ends with lgkmcnt(0) and every DMA lands in a stage whose last readers
//   finished at least one barrier earlier (the refills never race a read).
// BM = 192 (cfg 16): 96 rows per group, the same schedule with 3 A pieces per lane — 226 tiles for
// conv5's 43264 x 256 output fill one round of 256 CUs where 256-row tiles leave 87 CUs idle.
template <int BM, int BN>
__global__ void __launch_bounds__(512) conv_bf16_pp_kernel(ArgsW a) {
  constexpr int HM = BM / 2, TM = HM / 16, WN = BN / 4, TN = WN / 16;  // HM: a group's A rows
  constexpr int SZ = BM * kBK;       // bf16 per A stage
  constexpr int SB = BN * kBK;       // bf16 per B stage
  constexpr int NA = HM / 32, NB = BN / 64;  // DMA pieces per lane per K tile: this group's A rows, B half
  static_assert(HM % 32 == 0, "a group's rows are whole 32-row DMA blocks");
  static_assert(TN >= 1 && NB >= 1, "tile split");
  constexpr int CH = BN / 8, EW = BN + 8;  // epilogue image rows padded by 16 B (conflict-free)
  extern __shared__ __attribute__((aligned(16))) bf16 lds_b[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA M0 values stay scalar
  const int G = __builtin_amdgcn_readfirstlane(wave >> 2);  // wave-uniform, scalar
  const int wl = wave & 3, tl = tid & 255, wn = wave & 3, g = blockIdx.z;
  int tile;
  {
    const int nwg = gridDim.x, b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int mt = tile / a.n_ntiles, nt = tile - mt * a.n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const bf16* x = a.x + g * a.Cg;
  const bf16* wg = a.w + static_cast<size_t>(g) * a.kpad_n * a.kpad;
  // this lane's 4 A rows and 4 B rows: row G*128 + j*32 + tl/8, physical chunk tl&7 holding logical u
  const int u = (tl & 7) ^ ((tl >> 4) & 7);
  int aoff[NA], boff[NB];  // 32-bit element offsets from the (scalar) x / wg bases: fewer VGPRs
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = G * HM + j * 32 + (tl >> 3);
    const int m = m0 + row;
    int o = 0;
    if (m < a.M) {
      const int n = m / a.HoWo, rr = m - n * a.HoWo, oy = rr / a.Wo, ox = rr - oy * a.Wo;
      o = ((n * a.Hp + oy * a.S) * a.Wp + ox * a.S) * a.C;
    }
    aoff[j] = o;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)  // B row G*BN/2 + j*32 + tl/8 (< 2^31: packed weights of one group)
    boff[j] = min(n0 + G * (BN / 2) + j * 32 + (tl >> 3), a.kpad_n - 1) * a.kpad + u * 8;
  const int T = a.ktiles;
  int uc, ufw, ufh;  // the lane's K unit as (filter row, column, channel), advanced per A issue
  {
    const int k = u * 8, tap = k / a.Cg;
    uc = k - tap * a.Cg;
    ufh = tap / a.F;
    ufw = tap - ufh * a.F;
  }
  lds_b16* lds3 = (lds_b16*)(lds_b);
  const int drow = (G * HM + wl * 8) * kBK;  // this wave's first A DMA row (+ j*32 rows)
  const int dbrow = (G * (BN / 2) + wl * 8) * kBK;  // ... and B row
  auto issueA = [&](int st) {  // the next K tile of this group's A rows (issued in K order)
    const int ko = ufh < a.F ? (ufh * a.Wp + ufw) * a.C + uc : 0;
    uc += kBK;
    while (uc >= a.Cg) {
      uc -= a.Cg;
      if (++ufw == a.F) {
        ufw = 0;
        ++ufh;
      }
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) glds16(x + (aoff[j] + ko), lds3 + st * SZ + drow + j * 32 * kBK);
  };
  auto issueB = [&](int kt, int st) {
#pragma unroll
    for (int j = 0; j < NB; ++j) glds16(wg + (boff[j] + kt * kBK), lds3 + 2 * SZ + st * SB + dbrow + j * 32 * kBK);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int hq = lane >> 4, sw = (lane >> 1) & 7;
  const int arow = (G * HM + (lane & 15)) * kBK, brow = (wn * WN + (lane & 15)) * kBK;

  // prologue: tile 0 (both groups' halves), and G1's B_1
  issueA(0);
  issueB(0, 0);
  if (G == 1 && T > 1) issueB(1, 1);
  if (G == 1 && T > 1)
    lds_barrier<NB>();  // #0
  else
    lds_barrier<0>();
  if (G == 1) lds_barrier<>();  // the stagger
  asm volatile("" ::: "memory");
  int sb = 0;  // B stage of tile t (t % 3)
  for (int t = 0; t < T; ++t) {
    // ---- L_t: fragments of tile t, then this group's refills ----
    const bf16* A = lds_b + (t & 1) * SZ;
    const bf16* B = lds_b + 2 * SZ + sb * SB;
    bf16x8 a0[TM], b0[TN], a1[TM], b1[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(B + brow + j * 16 * kBK + (hq ^ sw) * 8);
#pragma unroll
    for (int i = 0; i < TM; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(A + arow + i * 16 * kBK + (hq ^ sw) * 8);
#pragma unroll
    for (int j = 0; j < TN; ++j) b1[j] = *reinterpret_cast<const bf16x8*>(B + brow + j * 16 * kBK + ((4 + hq) ^ sw) * 8);
#pragma unroll
    for (int i = 0; i < TM; ++i)
      a1[i] = *reinterpret_cast<const bf16x8*>(A + arow + i * 16 * kBK + ((4 + hq) ^ sw) * 8);
    __builtin_amdgcn_sched_barrier(0);
    const int s1 = sb == 2 ? 0 : sb + 1, s2 = s1 == 2 ? 0 : s1 + 1;
    if (G == 0) {
      if (t + 1 < T) {
        issueA((t + 1) & 1);
        issueB(t + 1, s1);
      }
    } else {
      if (t + 1 < T) issueA((t + 1) & 1);
      if (t + 2 < T) issueB(t + 2, s2);
      if (t + 2 < T)  // retire B_{t+1} (issued one L section earlier) before the barrier
        wait_vm<NA + NB>();
      else if (t + 1 < T)
        wait_vm<NA>();
      else
        wait_vm<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier<>();
    asm volatile("" ::: "memory");
    // ---- M_t ----
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a0[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a1[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (G == 0) {
      if (t + 1 < T)
        lds_barrier<0>();  // this group's A_{t+1}, B_{t+1}
      else
        lds_barrier<>();
    } else {
      if (t + 2 < T)  // A_{t+1} (B_{t+2} may fly)
        lds_barrier<NB>();
      else
        lds_barrier<0>();
    }
    asm volatile("" ::: "memory");
    sb = s1;
  }
  if (G == 0) lds_barrier<>();  // balance the stagger: every wave is past its last read
  asm volatile("" ::: "memory");

  // epilogue (as conv_bf16_big_kernel): the padded tile image (132 KiB) from the LDS base, ooff in
  // the last KiB
  int* ooff_s = reinterpret_cast<int*>(lds_b + 2 * SZ + 3 * SB - 512);
  static_assert(BM * EW + 512 <= 2 * SZ + 3 * SB, "epilogue image + offsets fit the stages");
  if (tid < BM) {
    const int m = m0 + tid;
    int oo = -1;
    if (m < a.M) {
      const int n = m / a.HoWo, rr = m - n * a.HoWo, oy = rr / a.Wo, ox = rr - oy * a.Wo;
      oo = ((n * a.Hb + oy + a.h_off) * a.Wb + ox + a.w_off) * a.Cb + a.c_off;
    }
    ooff_s[tid] = oo;
  }
  bf16* E = lds_b;
  using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
  const int mcol = lane & 15;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WN + j * 16 + hq * 4, f = n0 + nl;
    const f32x4 bv = (a.bias && f < a.Kg) ? *reinterpret_cast<const f32x4*>(a.bias + g * a.Kg + f) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = G * HM + i * 16 + mcol;
      f32x4 v = acc[i][j] + bv;
      if (a.relu) v = f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
      *reinterpret_cast<bf16x4*>(E + ml * EW + nl) =
          bf16x4{static_cast<bf16>(v.x), static_cast<bf16>(v.y), static_cast<bf16>(v.z), static_cast<bf16>(v.w)};
    }
  }
  __syncthreads();
  bf16* out = a.out + g * a.Kg;
  for (int q = tid; q < BM * CH; q += 512) {
    const int ml = q / CH, c = q - ml * CH;
    const int o = ooff_s[ml], f = n0 + c * 8;
    if (o >= 0 && f < a.Kg)
      *reinterpret_cast<u32x4*>(out + o + f) = *reinterpret_cast<const u32x4*>(E + ml * EW + c * 8);
  }
}

struct BigCfg {
  int BM, BN, threads, nst;
  int wgs_per_cu;  // co-resident workgroups (LDS / registers)
  float eff;       // relative per-CU MFMA efficiency (anx_bf16bench, 256 images)
};
// eff: cfg 2 vs 4 and 0 vs 4 are set so the ceil-rounds model ranks them as measured (conv1p:
// 128x96 ahead of 256x96; conv5, 169 256x256 tiles in one partial round: 256x256 ahead of 1014
// 128x96 tiles in two). The 3-stage configs ran 0.55-0.8 of cfg 0 on conv2-5 (deeper prefetch does
// not pay where a K tile's MFMA work already covers the DMA, and it takes the LDS a second 128-row
// workgroup per CU would use): they serve the FC layers. 9-11: cfgs 0, 3, 4 without PIPE (A/B).
constexpr BigCfg kCfg[] = {{256, 256, 512, 2, 1, 1.0f},  {256, 128, 512, 2, 1, 0.86f}, {256, 96, 512, 2, 1, 0.7f},
                           {128, 128, 256, 2, 2, 0.92f}, {128, 96, 256, 2, 2, 0.74f},  {256, 128, 512, 3, 1, 0.7f},
                           {128, 128, 256, 3, 1, 0.6f},  {128, 96, 256, 3, 1, 0.5f},   {256, 64, 512, 3, 1, 0.6f},
                           {256, 256, 512, 2, 1, 0.5f},  {128, 128, 256, 2, 2, 0.5f},  {128, 96, 256, 2, 2, 0.5f},
                           {256, 256, 512, 0, 1, 1.04f},   // 12: ping-pong (A 2 + B 3 stages): 2-7 % over 0
                           {256, 128, 512, 0, 1, 0.8f},    // 13: ping-pong 256x128 (conv3/4: 90 / 125 us vs 77 / 109 for cfg 3)
                           {96, 96, 256, 2, 3, 0.8f},      // 14: 96x96, 3 workgroups/CU (short-K conv1p: 101 vs 109 us for cfg 4)
                           {64, 96, 256, 2, 3, 0.6f},      // 15: 64x96, 3 workgroups/CU
                           {192, 256, 512, 0, 1, 1.0f}};   // 16: ping-pong 192x256 (conv5: one round of 226 tiles)
constexpr int kNumCfg = sizeof(kCfg) / sizeof(kCfg[0]);
// (Round 5: the activation-streaming FC kernel, activations global -> VGPR four K tiles ahead, was
// removed: slower than the wide-tile split-K FC at every layer, profiles/r02_bf16bench_fc_b256.txt.)


size_t lds_bytes(const BigCfg& c) {
  if (c.nst == 0) return (static_cast<size_t>(2) * c.BM + 3 * c.BN) * kBK * 2;  // ping-pong: A x 2 + B x 3 stages
  return static_cast<size_t>(c.nst) * (c.BM + c.BN) * kBK * 2 + static_cast<size_t>(c.BM) * 4;
}

}  // namespace

static_assert(kNumCfg == kConvBf16BigCfgs, "bf16_ops.hpp: kConvBf16BigCfgs");
int conv_bf16_big_cfgs() { return kNumCfg; }

bool conv_bf16_big_ok(const ConvPlanB& p, int cfg, const OutViewB& out) {
  if (cfg < 0 || cfg >= kNumCfg) return false;
  return p.vec8 && !p.taps8 && p.Kg % 8 == 0 && out.Cb % 8 == 0 && out.c_off % 8 == 0 && out.base &&
         lds_bytes(kCfg[cfg]) <= 160 * 1024 && static_cast<long>(p.N) * p.Hp * p.Wp * p.C < (1L << 31) &&
         static_cast<long>(p.N) * out.Hb * out.Wb * out.Cb < (1L << 31);
}

// Wave-quantization cost model: a config's time ~ rounds of co-resident workgroups x tile area x
// workgroups per CU / efficiency (ceil, so a 1.3-round launch costs 2 rounds); ties keep the
// lower config index.
int pick_bf16_big_cfg(const ConvPlanB& p, const OutViewB& out, int cus) {
  const long M = static_cast<long>(p.N) * p.Ho * p.Wo;
  int best = -1;
  double best_cost = 0;
  for (int c = 0; c < kNumCfg; ++c) {
    if (!conv_bf16_big_ok(p, c, out)) continue;
    const BigCfg& k = kCfg[c];
    const long tiles = (M + k.BM - 1) / k.BM * ((p.Kg + k.BN - 1) / k.BN) * p.groups;
    const long slots = static_cast<long>(cus) * k.wgs_per_cu;
    const long rounds = (tiles + slots - 1) / slots;
    const double cost = static_cast<double>(rounds) * k.BM * k.BN * k.wgs_per_cu / k.eff;
    if (best < 0 || cost < best_cost * 0.999) {
      best = c;
      best_cost = cost;
    }
  }
  return best;
}

// Fully-connected layers (M = batch, 1x1): 256-row tiles (the whole batch at 256: each weight tile
// streamed once) x 64 columns over 8 waves with 3 LDS stages (cfg 8), K split so that tiles x
// slices ~ one workgroup per CU with >= 4 K tiles per slice. Measured at 256 images
// (profiles/r02_bf16bench_b256.txt): FC6 36 us, FC7 23 us, FC8 18 us with the reduce, against 43 /
// 28 / 24 us for the 128x128 split-K path.
BigFc pick_bf16_big_fc(const ConvPlanB& p, int cus, int cfg, int min_kt) {
  BigFc r{-1, 1};
  if (p.Ho != 1 || p.Wo != 1 || p.groups != 1 || p.Kg % 8) return r;
  const OutViewB probe{reinterpret_cast<__bf16*>(16), 1, 1, p.Kg, 0, 0, 0};
  // forced configs (knob bf16_fc_cfg, A/B): any slab-capable wide-tile config (not the ping-pong
  // kernels), K split at most kMaxFcSplit ways (the engine's slab workspace is sized for that)
  r.cfg = cfg >= 0 && cfg != 12 && cfg != 13 && cfg != 16 ? cfg : 8;
  if (!conv_bf16_big_ok(p, r.cfg, probe)) return BigFc{-1, 1};
  const BigCfg& c = kCfg[r.cfg];
  const long tiles = (p.N + c.BM - 1) / c.BM * ((p.Kg + c.BN - 1) / c.BN);
  const int ktiles = p.kpad / kBK;
  const long want = (static_cast<long>(cus) * c.wgs_per_cu + tiles - 1) / tiles;
  r.ksplit = static_cast<int>(
      std::max<long>(1, std::min<long>({want, ktiles / std::max(1, min_kt), static_cast<long>(kMaxFcSplit)})));
  return r;
}

hipError_t conv2d_bf16_big(const ConvPlanB& p, int cfg, const void* x, const void* wpacked, const int* koff,
                           const float* bias, OutViewB out, bool relu, hipStream_t s, SplitK split) {
  if (!conv_bf16_big_ok(p, cfg, out)) return hipErrorInvalidValue;
  const int ksplit = std::max(1, split.ksplit);
  const bool slab = split.ws != nullptr;  // fp32 slabs (also at ksplit 1: an fp32 result via the reduce)
  if ((cfg == 12 || cfg == 13 || cfg == 16) && slab) cfg = cfg == 13 ? 1 : 0;  // ping-pong: no split-K slab epilogue
  if ((ksplit > 1 && !slab) || (slab && p.groups != 1)) return hipErrorInvalidValue;
  const long M = static_cast<long>(p.N) * p.Ho * p.Wo;
  if (M == 0) return hipSuccess;
  const BigCfg c = kCfg[cfg];
  ArgsW a{};
  a.x = static_cast<const bf16*>(x);
  a.w = static_cast<const bf16*>(wpacked);
  a.koff = koff;
  a.bias = bias;
  a.out = out.base;
  a.M = static_cast<int>(M);
  a.HoWo = p.Ho * p.Wo;
  a.Wo = p.Wo;
  a.Hp = p.Hp;
  a.Wp = p.Wp;
  a.C = p.C;
  a.S = p.S;
  a.F = p.F;
  a.Cg = p.Cg;
  a.Kg = p.Kg;
  a.kpad = p.kpad;
  a.kpad_n = p.kpad_n;
  a.ktiles = p.kpad / kBK;
  a.n_ntiles = (p.Kg + c.BN - 1) / c.BN;
  a.m_tiles = static_cast<int>((M + c.BM - 1) / c.BM);
  a.Hb = out.Hb;
  a.Wb = out.Wb;
  a.Cb = out.Cb;
  a.h_off = out.h_off;
  a.w_off = out.w_off;
  a.c_off = out.c_off;
  a.relu = relu ? 1 : 0;
  a.kt_per = (a.ktiles + ksplit - 1) / ksplit;
  a.ws = split.ws;
  const dim3 grid(static_cast<unsigned>(a.m_tiles * a.n_ntiles), ksplit, p.groups);
  const size_t lds = lds_bytes(c);
#define ANX_BIG_CFGS(X)         \
  X(0, 256, 256, 2, 4, 2, true)        \
  X(1, 256, 128, 4, 2, 2, false)       \
  X(2, 256, 96, 4, 2, 2, false)        \
  X(3, 128, 128, 2, 2, 2, true)        \
  X(4, 128, 96, 2, 2, 2, true)         \
  X(5, 256, 128, 4, 2, 3, false)       \
  X(6, 128, 128, 2, 2, 3, false)       \
  X(7, 128, 96, 2, 2, 3, false)        \
  X(8, 256, 64, 8, 1, 3, false)     \
  X(9, 256, 256, 2, 4, 2, false)    \
  X(10, 128, 128, 2, 2, 2, false)   \
  X(11, 128, 96, 2, 2, 2, false)   \
  X(14, 96, 96, 2, 2, 2, true)      \
  X(15, 64, 96, 2, 2, 2, true)
  static const hipError_t attr = [] {
#define ANX_ATTR(I, BM, BN, WGM, WGN, NST, P)                                                                     \
  for (const void* k : {reinterpret_cast<const void*>(conv_bf16_big_kernel<BM, BN, WGM, WGN, NST, false, P>),    \
                        reinterpret_cast<const void*>(conv_bf16_big_kernel<BM, BN, WGM, WGN, NST, true, P>)}) {  \
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);     \
    if (e != hipSuccess) return e;                                                                            \
  }
    ANX_BIG_CFGS(ANX_ATTR)
#undef ANX_ATTR
    return hipSuccess;
  }();
  if (attr != hipSuccess) return attr;
  if (cfg == 12 || cfg == 13 || cfg == 16) {
    static const hipError_t pattr = [] {
      for (const void* k : {reinterpret_cast<const void*>(conv_bf16_pp_kernel<256, 256>),
                            reinterpret_cast<const void*>(conv_bf16_pp_kernel<256, 128>),
                            reinterpret_cast<const void*>(conv_bf16_pp_kernel<192, 256>)}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    }();
    if (pattr != hipSuccess) return pattr;
    if (cfg == 12)
      conv_bf16_pp_kernel<256, 256><<<grid, 512, lds, s>>>(a);
    else if (cfg == 13)
      conv_bf16_pp_kernel<256, 128><<<grid, 512, lds, s>>>(a);
    else
      conv_bf16_pp_kernel<192, 256><<<grid, 512, lds, s>>>(a);
    return hipGetLastError();
  }
  switch (cfg) {
#define ANX_CASE(I, BM, BN, WGM, WGN, NST, P)                                                \
  case I:                                                                                    \
    if (slab)                                                                                \
      conv_bf16_big_kernel<BM, BN, WGM, WGN, NST, true, P><<<grid, c.threads, lds, s>>>(a);  \
    else                                                                                     \
      conv_bf16_big_kernel<BM, BN, WGM, WGN, NST, false, P><<<grid, c.threads, lds, s>>>(a); \
    break;
    ANX_BIG_CFGS(ANX_CASE)
#undef ANX_CASE
    default:
      return hipErrorInvalidValue;
  }
#undef ANX_BIG_CFGS
  return hipGetLastError();
}

}  // namespace anx::hip
