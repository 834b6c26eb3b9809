// Fused Winograd F(4x4,5x5) batched GEMM + output transform for Conv2, fp32 on v_mfma_f32_16x16x4_f32
// (included by wino_gemm.hip and by the anx_wgemm A/B tool).
//
// Why a second tile size: F(3x3,5x5) spends 49 transform points on 9 outputs (5.44 multiplies per
// output), F(4x4,5x5) 64 on 16 (4.0): Conv2's 27x27 map is 81 tiles of 3x3 but 49 tiles of 4x4 (one
// wasted row and column), so the MFMA work per image drops from 195 to 154 MFLOP (-21 %) and V from
// 1.52 to 1.20 MB per image. Its fp32 error is 6.8e-7 of sum|x*w| against 5.2e-7 for F(3,5)
// (tools/winograd_numerics.py; points {0, +-1, +-2, +-1/2, inf}).
//
// The price is the output fold: 16 outputs per tile. The 3x3 kernel's wave tile (32 tiles x 32 filters
// on 32x32x2 MFMAs) would need 16 x 16 = 256 fold registers per lane, so this kernel runs 32 tiles x 16
// filters per wave on 16x16x4 MFMAs (same f32 rate: 64 FLOP per cycle per SIMD): two 16x16 blocks share
// each B fragment, the fold holds Y[16 outputs][8 values] = 128 registers, and every point folds
// 128 FMAs (2.7 per MFMA) behind the next point's MFMAs.
//
// Everything else is wino_gemm.hpp's schedule: an NST-slot LDS ring of BK-channel slices filled by
// buffer_load ... lds (1 KiB per wave instruction, swizzled source offsets), one barrier per slice,
// compile-time slot / offset / wait counts in a UP-point loop body with a peeled tail, fold pinned
// behind the MFMAs with sched_group_barrier, bias + ReLU + NHWC store once at the end through an LDS
// transpose (16-B stores).
//
// Fragment reads: 16x16x4 takes one A and one B value per lane, lane l = (row l % 16, k-group l / 16).
// A lane's ds_read_b128 of unit 4s + l/16 of its row yields 4 channels, one per k-step: k-step j of
// channel group s multiplies channel 16s + 4(l/16) + j (the same permutation on A and B, so the sum is
// unchanged). The LDS swizzle (swz16) makes every ds_read_b128 lane group hit 16 distinct 16-B slots.
//
// Reference op: convKernel (v3_cuda_only/src/layers_cuda.cu:20-46), one thread per output.
#pragma once
#include "wino_gemm.hpp"

#include "anx/winograd_f45.hpp"

namespace anx::hip::wg16 {

using wg::f32x4;
using wg::lds_f32;
using wg::lds_void;
using wg::static_for;

struct Coef64 {
  float v[64][16];
};
constexpr Coef64 make_coef64() {
  Coef64 t{};
  for (int ab = 0; ab < 64; ++ab)
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) t.v[ab][i * 4 + j] = wino45::kAT[i][ab / 8] * wino45::kAT[j][ab % 8];
  return t;
}
static __constant__ Coef64 c_coef64 = make_coef64();

#include "wino_gemm16_sched.inc"

// LDS swizzle of the 16-B unit u of row r: u ^ swz16(r). ds_read_b128 is served in four 16-lane groups,
// {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32 (MI355X_MICROARCH.md, LDS): with 48-float rows
// a group's (row, unit) pairs land on 16 distinct 16-B slots iff the XOR of rows 0-3 / 4-7 / 8-11 / 12-15
// is 0 / 2 / 3 / 1 (the 3x3 kernel's (r >> 2) & 3 left every group 2-way conflicted here: 49 % of this
// kernel's LDS cycles, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/r05_f45/pmc_summary_lane1.md).
// tools/lds_swizzle_check.py checks both tables against that lane-group model.
template <int U4>
__device__ __forceinline__ int swz16(int row) {
  if constexpr (U4 == 12)
    return (0x78 >> (2 * ((row >> 2) & 3))) & 3;
  else if constexpr (U4 == 24)
    // 96-float rows (24 units): a row starts at slot 8 * (row & 1) mod 16, and a lane group reads unit 4s + kg
    // of rows r16 with kg in {0,1} (or {2,3}). Within each row parity the group's 8 lanes must cover the 8
    // low-3-bit values: XOR {0,2,4,6} over rows {0,2,12,14} and again over {4,6,8,10} (their kg differs by one,
    // flipping bit 0), the same for the odd rows. Round 5's table (0x13dd90722a48) left every group 2-way
    // conflicted (SQ_LDS_BANK_CONFLICT 49 % of SQ_LDS_IDX_ACTIVE, profiles/r05_f45/wg45_pmc_waits.md).
    return (row & 2) | ((row >> 1) & 4);
  else
    return wg::swz<U4>(row);
}

// WM x WN waves of 16 NB tiles x 16 filters (NB 16x16 MFMA blocks sharing each B fragment); BK-channel
// slices through an NST-slot ring.
template <int WM_, int WN_, int BK_, int NST_, int NB_ = 2>
struct Cfg {
  static constexpr int NB = NB_;
  static constexpr int NPT = 64, C = 96, NQ = 16, NE = 4 * NB;  // points, channels, outputs, values per lane
  static constexpr int WM = WM_, WN = WN_, BK = BK_, NST = NST_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = 16 * NB * WM, BN = 16 * WN, U4 = BK / 4;
  static constexpr int KS = C / BK, TOTAL = NPT * KS;
  static constexpr int A_INS = BM * U4 / 64, B_INS = BN * U4 / 64;
  static constexpr int A_MAX = (A_INS + NW - 1) / NW, B_MAX = (B_INS + NW - 1) / NW;
  static constexpr int PW_MIN = A_INS / NW + B_INS / NW;
  static constexpr int A_FL = BM * BK, STAGE = (BM + BN) * BK;
  static constexpr size_t kLdsBytes = static_cast<size_t>(NST) * STAGE * sizeof(float);
  static constexpr int UP = wg::even_up(KS, NST);
  static constexpr int NI = (TOTAL + 1 - NST) / (UP * KS);
  static constexpr int TAIL = NPT - NI * UP;
  static constexpr int G4 = BK / 16;     // 16-channel groups per slice (one ds_read_b128 per operand row each)
  static constexpr int MF = BK / 4 * NB;  // MFMAs per slice (k-steps x row blocks)
  static constexpr int NF = NQ * NE;     // fold FMAs per point
  // workgroups per CU the VGPR budget is sized for: 8 waves per CU with 2 blocks per wave (Y = 128
  // registers), 16 with one (Y = 64: 4 waves per SIMD)
  static constexpr int MINB = (NB == 2 ? 8 : 16) / NW >= 1 ? (NB == 2 ? 8 : 16) / NW : 1;
  static_assert(C % BK == 0 && BK % 16 == 0 && A_INS * 64 == BM * U4 && B_INS * 64 == BN * U4, "tile shape");
  static_assert(U4 == 4 || U4 == 8 || U4 == 12 || U4 == 24, "swizzle defined for 4, 8, 12, 24 units per row");
  static_assert(NST >= 2 && NI >= 1 && TAIL >= 1, "ring / loop shape");
  static_assert(NB == 1 || NB == 2, "one or two 16-tile blocks per wave");
};

// ABL: bit0 no fold, bit1 no DMA refills, bit2 no barrier, bit4 no sched_group_barrier pinning, bit5 no
// epilogue stores (cost probes, A/B tool only); bit6 the hand-scheduled slice (wino_gemm16_sched.inc, knob
// conv2_sched): fragment reads two groups ahead with counted waits, alternating accumulators, fold FMAs
// behind every MFMA. Bitwise identical to the compiler-scheduled kernel.
template <class G, int ABL, bool POOL = false>
__global__ void __launch_bounds__(G::NT, G::MINB) gemm16_kernel(wg::Args a) {
  constexpr int KS = G::KS, BK = G::BK, NW = G::NW, NST = G::NST, U4 = G::U4, MF = G::MF, G4 = G::G4, NF = G::NF;
  constexpr bool kFold = !(ABL & 1), kDma = !(ABL & 2), kBar = !(ABL & 4), kPin = !(ABL & 16), kStore = !(ABL & 32);
  constexpr bool kAsm = (ABL & 64) != 0;
  static_assert(!kAsm || (G::G4 == 6 && G::NB == 2 && G::KS == 1 && G::NQ == 16 && G::NE == 8),
                "the hand-scheduled slice is generated for one 96-channel point per slice, two 16x16 blocks");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % G::WM, wn = wave / G::WM;
  // XCD-aware order (as wino_gemm.hpp): the n_ntiles workgroups reading one V slab share blockIdx.x % 8
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles, pt = (jb / a.n_ntiles) * 8 + xcd;
  if (pt >= a.n_ptiles) return;  // whole workgroup, before any DMA or barrier
  const int p0 = pt * G::BM, n0 = nt * G::BN;

  int voff[G::A_MAX], uoff[G::B_MAX];
#pragma unroll
  for (int i = 0; i < G::A_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::A_INS ? q : 0) * 64 + lane;
    const int row = U / U4, u = (U - row * U4) ^ swz16<U4>(row);
    const int p = p0 + row;
    voff[i] = ((p < a.P ? p : 0) * G::NPT * a.vct + 4 * u) * 4;  // rows past P read tile 0, never stored
  }
#pragma unroll
  for (int i = 0; i < G::B_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::B_INS ? q : 0) * 64 + lane;
    const int row = U / U4, u = (U - row * U4) ^ swz16<U4>(row);
    uoff[i] = ((n0 + row) * G::C + 4 * u) * 4;
  }
#if __HIP_DEVICE_COMPILE__
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.V), 0, a.vbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
#endif
  [[maybe_unused]] lds_f32* lds3 = (lds_f32*)(lds);
  auto issue = [&](int ab, int ks, int slot) {
    if constexpr (kDma) {
#if __HIP_DEVICE_COMPILE__
      lds_f32* st = lds3 + slot * G::STAGE;
      const int vso = (ab * a.vct + ks * BK) * 4;
      const int uso = (ab * a.u_rows * G::C + ks * BK) * 4;
#pragma unroll
      for (int i = 0; i < G::A_MAX; ++i)
        if ((G::A_INS % NW == 0) || wave + NW * i < G::A_INS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (lds_void*)(st + (wave + NW * i) * 256), 16, voff[i], vso, 0, 0);
#pragma unroll
      for (int i = 0; i < G::B_MAX; ++i)
        if ((G::B_INS % NW == 0) || wave + NW * i < G::B_INS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)(st + G::A_FL + (wave + NW * i) * 256), 16, uoff[i],
                                                   uso, 0, 0);
#endif
    }
  };

  const int r16 = lane & 15, kg = lane >> 4;
  // byte addresses (slot 0) of my rows' fragment units: A rows wm*32 + r16 (+16), B row wn*16 + r16
  int ra0[G4], ra1[G4], rb[G4];
#pragma unroll
  for (int s = 0; s < G4; ++s) {
    const int u = 4 * s + kg, x0 = wm * 16 * G::NB + r16, x1 = x0 + 16, y = wn * 16 + r16;
    ra0[s] = (x0 * BK + 4 * (u ^ swz16<U4>(x0))) * 4;
    ra1[s] = (x1 * BK + 4 * (u ^ swz16<U4>(x1))) * 4;
    rb[s] = (G::A_FL + y * BK + 4 * (u ^ swz16<U4>(y))) * 4;
  }

  float Y[G::NQ][G::NE];  // Y[q][e]: output q of accumulator value e (block e >> 2, register e & 3)
#pragma unroll
  for (int q = 0; q < G::NQ; ++q)
#pragma unroll
    for (int e = 0; e < G::NE; ++e) Y[q][e] = 0.f;
  f32x4 acc[2][2] = {};  // [point parity][row block]
  float cq[2][G::NQ];

  auto frag = [&](int addr) { return *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(lds) + addr); };
  auto fold_one = [&](auto J, auto FI) {
    constexpr int j = decltype(J)::value, fi = decltype(FI)::value, q = j / G::NE, e = j % G::NE;
    Y[q][e] = __builtin_fmaf(cq[fi][q], acc[fi][e >> 2][e & 3], Y[q][e]);
  };

  auto slice = [&](int pb, auto LIT, auto ABS, auto FOLD) {
    constexpr int lit = decltype(LIT)::value;
    constexpr bool abs_it = decltype(ABS)::value, fold = decltype(FOLD)::value && kFold;
    constexpr int ks = lit % KS, ai = (lit / KS) & 1, slot = lit % NST, nlit = lit + NST - 1;
    constexpr bool refill = !abs_it || nlit < G::TOTAL;
    constexpr int ahead = abs_it ? ((G::TOTAL - 1 - lit) < NST - 2 ? (G::TOTAL - 1 - lit) : NST - 2) : NST - 2;
    const int ab = pb + lit / KS;
    __builtin_amdgcn_sched_barrier(0);
    constexpr int vm = kDma ? ahead * G::PW_MIN : 0;
    if constexpr (kBar)
      lds_barrier<vm>();
    else
      wg::wait_vm_lgkm<vm>();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if constexpr (refill && !(kAsm && ((ABL >> 10) & 3) != 0)) issue(pb + nlit / KS, nlit % KS, nlit % NST);
    auto load_coef = [&] {
      const float* cr = c_coef64.v[ab];
#pragma unroll
      for (int q = 0; q < G::NQ; ++q) cq[ai][q] = cr[q];
    };
    if constexpr (kAsm && fold) {
      // the hand-scheduled slice reads the previous point's coefficients: make the compiler's wait for
      // their scalar load land here, behind the barrier that already drained it, and not after the next
      // point's load (it cannot see the barrier's lgkmcnt(0) and would wait for both)
      asm volatile("" ::"s"(cq[ai ^ 1][0]), "s"(cq[ai ^ 1][1]), "s"(cq[ai ^ 1][2]), "s"(cq[ai ^ 1][3]),
                   "s"(cq[ai ^ 1][4]), "s"(cq[ai ^ 1][5]), "s"(cq[ai ^ 1][6]), "s"(cq[ai ^ 1][7]), "s"(cq[ai ^ 1][8]),
                   "s"(cq[ai ^ 1][9]), "s"(cq[ai ^ 1][10]), "s"(cq[ai ^ 1][11]), "s"(cq[ai ^ 1][12]),
                   "s"(cq[ai ^ 1][13]), "s"(cq[ai ^ 1][14]), "s"(cq[ai ^ 1][15]));
    }
    if constexpr (ks == 0) load_coef();
    constexpr int so = slot * G::STAGE * 4;
    if constexpr (kAsm) {
      constexpr int mode = (ABL >> 7) & 3, dm = refill ? (ABL >> 10) & 3 : 0;
      constexpr bool pk = (ABL & 512) != 0;
      static_assert((mode == 0 && !pk) || (mode == 1 && pk) || (mode == 2 && pk), "generated fold forms");
      [[maybe_unused]] Dma d;
      if constexpr (dm != 0) {
        static_assert(G::A_MAX == 3 && G::B_MAX == 6 && G::A_INS % NW == 0 && G::B_INS % NW == 0, "DMA shape");
        const int abn = pb + nlit / KS;
#pragma unroll
        for (int i = 0; i < 3; ++i) d.voff[i] = voff[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) d.uoff[i] = uoff[i];
#if __HIP_DEVICE_COMPILE__
        d.vr = vr;
        d.ur = ur;
#endif
        d.vso = (abn * a.vct) * 4;
        d.uso = (abn * a.u_rows * G::C) * 4;
        d.wb = static_cast<int>(reinterpret_cast<size_t>(lds3)) + wave * 1024;  // LDS byte address of my pieces
      }
      constexpr int rs = (nlit % NST) * G::STAGE * 4;
      auto& a0 = acc[ai][0];
      auto& a1 = acc[ai][1];
      if constexpr (fold) {
        const auto& p0 = acc[ai ^ 1][0];
        const auto& p1 = acc[ai ^ 1][1];
        const auto& c = cq[ai ^ 1];
#define ANX_WG16_FOLD(F)                                                      \
  if constexpr (dm == 0) F##_d0<so>(Y, a0, a1, p0, p1, c, ra0, ra1, rb);      \
  if constexpr (dm == 1) F##_d1<so, rs>(Y, a0, a1, p0, p1, c, ra0, ra1, rb, d); \
  if constexpr (dm == 2) F##_d2<so, rs>(Y, a0, a1, p0, p1, c, ra0, ra1, rb, d); \
  if constexpr (dm == 3) F##_d3<so, rs>(Y, a0, a1, p0, p1, c, ra0, ra1, rb, d);
        if constexpr (mode == 0) { ANX_WG16_FOLD(slice_fold0) }
        if constexpr (mode == 1) { ANX_WG16_FOLD(slice_fold1p) }
        if constexpr (mode == 2) { ANX_WG16_FOLD(slice_fold2p) }
#undef ANX_WG16_FOLD
      } else {
        if constexpr (dm == 0) slice_first_d0<so>(a0, a1, ra0, ra1, rb);
        if constexpr (dm == 1) slice_first_d1<so, rs>(a0, a1, ra0, ra1, rb, d);
        if constexpr (dm == 2) slice_first_d2<so, rs>(a0, a1, ra0, ra1, rb, d);
        if constexpr (dm == 3) slice_first_d3<so, rs>(a0, a1, ra0, ra1, rb, d);
      }
      if constexpr (decltype(FOLD)::value && !kFold)
        Y[0][0] += acc[ai ^ 1][0][0] + acc[ai ^ 1][G::NB - 1][0];  // probe: keep both blocks' MFMAs live
      return;
    }
    constexpr int j0 = NF * ks / KS, nj = NF * (ks + 1) / KS - j0;
    constexpr int NB = G::NB;
    f32x4 fa0[2], fa1[2], fb[2];
    fa0[0] = frag(ra0[0] + so);
    if constexpr (NB == 2) fa1[0] = frag(ra1[0] + so);
    fb[0] = frag(rb[0] + so);
    static_for<0, G4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      if constexpr (s + 1 < G4) {
        fa0[(s + 1) & 1] = frag(ra0[s + 1] + so);
        if constexpr (NB == 2) fa1[(s + 1) & 1] = frag(ra1[s + 1] + so);
        fb[(s + 1) & 1] = frag(rb[s + 1] + so);
      }
      static_for<0, 4>([&](auto K) {
        constexpr int k = decltype(K)::value, m = (s * 4 + k) * NB;
        constexpr bool first = ks == 0 && s == 0 && k == 0;
        acc[ai][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa0[s & 1][k], fb[s & 1][k], first ? f32x4{} : acc[ai][0], 0,
                                                          0, 0);
        if constexpr (fold)
          static_for<j0 + nj * m / MF, j0 + nj * (m + 1) / MF>(
              [&](auto J) { fold_one(J, std::integral_constant<int, ai ^ 1>{}); });
        if constexpr (NB == 2) {
          acc[ai][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa1[s & 1][k], fb[s & 1][k], first ? f32x4{} : acc[ai][1],
                                                            0, 0, 0);
          if constexpr (fold)
            static_for<j0 + nj * (m + 1) / MF, j0 + nj * (m + 2) / MF>(
                [&](auto J) { fold_one(J, std::integral_constant<int, ai ^ 1>{}); });
        }
      });
      if constexpr (kPin) {
        if constexpr (s + 1 < G4) __builtin_amdgcn_sched_group_barrier(0x100, 1 + NB, 0);  // the next group's reads
        static_for<0, 4 * NB>([&](auto M) {
          constexpr int m = s * 4 * NB + decltype(M)::value;
          constexpr int np = nj * (m + 1) / MF - nj * m / MF;  // fold FMAs behind this MFMA
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if constexpr (fold && np > 0) __builtin_amdgcn_sched_group_barrier(0x002, np, 0);
        });
      }
    });
    if constexpr (decltype(FOLD)::value && !kFold && ks == 0)
      Y[0][0] += acc[ai ^ 1][0][0] + acc[ai ^ 1][G::NB - 1][0];  // probe: keep both blocks' MFMAs live
  };
  using std::integral_constant;
  using T_ = integral_constant<bool, true>;
  using F_ = integral_constant<bool, false>;

  static_for<0, NST - 1>([&](auto IT) {
    constexpr int it = decltype(IT)::value;
    issue(it / KS, it % KS, it);
  });
  static_for<0, G::UP * KS>([&](auto IT) {
    constexpr int it = decltype(IT)::value;
    slice(0, IT, T_{}, integral_constant<bool, (it >= KS)>{});
  });
  for (int pb = G::UP; pb < G::NI * G::UP; pb += G::UP) {
    static_for<0, G::UP * KS>([&](auto LIT) { slice(pb, LIT, F_{}, T_{}); });
  }
  static_for<G::NI * G::UP * KS, G::TOTAL>([&](auto IT) { slice(0, IT, T_{}, T_{}); });
  // an MFMA's D read by a VALU: 12 wait states after the hand-scheduled slice's last MFMA (8-pass XDL)
  if constexpr (kAsm) asm volatile("s_nop 7\n\ts_nop 3" ::: "memory");
  static_for<0, NF>([&](auto J) { fold_one(J, integral_constant<int, (G::NPT - 1) & 1>{}); });

  // Epilogue: bias + ReLU, then per output q one LDS transpose of the wave's 32 tiles x 16 filters so each
  // lane stores a 16-B filter group. D layout (16x16x4): lane (r16, kg) holds filter n0 + wn*16 + r16 of
  // tiles wm*32 + 16*(e >> 2) + 4*kg + (e & 3).
  __syncthreads();  // the ring is idle (the last slice waited vmcnt(0)): reuse it as scratch
  const int fb = n0 + wn * 16;
  const float bv = a.bias ? a.bias[fb + r16] : 0.f;
  if constexpr (POOL) {
    // Pool2 (3x3 / 2 max) on 4x4 tiles: pooled pixel (2 ty + dy, 2 tx + dx) of tile t = (ty, tx) covers
    // rows 2 dy .. 2 dy + 2 and columns 2 dx .. 2 dx + 2 of the tile, i.e. its own rows 0-2 / 2-3 x columns
    // 0-2 / 2-3, plus column 0 of tile t + 1 (dx = 1), row 0 of tile t + tx (dy = 1) and position (0, 0) of
    // tile t + tx + 1 (both). A lane (filter r16) folds its 8 tiles' own parts in registers and posts the
    // five values its tiles give to their left / upper neighbours into a per-wave LDS image; the lane
    // owning a pixel's tile merges them. Neighbours past this workgroup's 32 tiles: the pixel is written
    // as a partial max, and the next workgroup writes its part to p2 (pool2_straddles; lrn_pooled_merge).
    constexpr int kCS = 5 * 16 + 4;  // floats per tile; + 4 puts the four kg lane groups on distinct banks
    static_assert(G::WM == 1 && G::NB == 2 && G::BM == kConv2PoolTiles, "pool2 epilogue: one wave row of 32 tiles");
    static_assert(G::kLdsBytes >= static_cast<size_t>(NW) * 32 * kCS * 4, "pool2 scratch");
    // LDS / global address spaces spelled out: with generic pointers every global store may alias the LDS
    // image, and the compiler serialises each pixel's LDS reads behind the previous pixel's store
    using gbl_f32 = __attribute__((address_space(1))) float;
    lds_f32* cb = lds3 + wave * 32 * kCS;
    float own[G::NE][4];
#pragma unroll
    for (int e = 0; e < G::NE; ++e) {
      float v[G::NQ];
#pragma unroll
      for (int q = 0; q < G::NQ; ++q) {
        v[q] = Y[q][e] + bv;
        if (a.relu) v[q] = fmaxf(v[q], 0.f);
      }
      float h0[4], h1[4];  // per row: columns 0-2, 2-3
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h0[r] = fmaxf(fmaxf(v[4 * r], v[4 * r + 1]), v[4 * r + 2]);
        h1[r] = fmaxf(v[4 * r + 2], v[4 * r + 3]);
      }
      own[e][0] = fmaxf(fmaxf(h0[0], h0[1]), h0[2]);
      own[e][1] = fmaxf(fmaxf(h1[0], h1[1]), h1[2]);
      own[e][2] = fmaxf(h0[2], h0[3]);
      own[e][3] = fmaxf(h1[2], h1[3]);
      lds_f32* c = cb + (16 * (e >> 2) + 4 * kg + (e & 3)) * kCS + r16;
      c[0] = fmaxf(fmaxf(v[0], v[4]), v[8]);  // column 0, rows 0-2: pixel (0, 1) of tile t - 1
      c[16] = fmaxf(v[8], v[12]);             // column 0, rows 2-3: pixel (1, 1) of tile t - 1
      c[32] = h0[0];                          // row 0, columns 0-2: pixel (1, 0) of tile t - tx
      c[48] = h1[0];                          // row 0, columns 2-3: pixel (1, 1) of tile t - tx
      c[64] = v[0];                           // (0, 0): pixel (1, 1) of tile t - tx - 1
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave, LDS in order: every lane's posts are visible
    const int ipt = a.ty * a.tx;
    gbl_f32* const pooled = (gbl_f32*)(a.out.base);
    gbl_f32* const p2 = (gbl_f32*)(a.p2);
    const int pc = a.out.Cb;  // channels per pooled pixel
    // tile t -> (image, tile row, tile column): one division per run of 4 consecutive tiles, then steps
    // (integer division is ~30 VALU instructions; 8 per lane cost the epilogue several us per launch)
    struct Pos {
      int n, y, x;
    };
    auto pos_of = [&](int t) {
      const int n = t / ipt, r = t - n * ipt, y = r / a.tx;
      return Pos{n, y, r - y * a.tx};
    };
    auto step = [&](Pos q) {  // the next tile in raster order
      if (++q.x == a.tx) {
        q.x = 0;
        if (++q.y == a.ty) q.y = 0, ++q.n;
      }
      return q;
    };
    Pos run[2] = {pos_of(p0 + 4 * kg), pos_of(p0 + 16 + 4 * kg)};
    float pix[G::NE][4];
#pragma unroll
    for (int e = 0; e < G::NE; ++e) {
      const int lt = 16 * (e >> 2) + 4 * kg + (e & 3), t = p0 + lt;
      const Pos ps = run[e >> 2];
      run[e >> 2] = step(ps);
      // the neighbours' posts, loaded unconditionally (tile index clamped into this wave's image) so the
      // 40 reads of a lane go out together behind one wait; -inf where the tile is another workgroup's
      const int j1 = lt + 1, j7 = lt + a.tx, j8 = j7 + 1;
      const lds_f32* c1 = cb + (j1 < 32 ? j1 : 31) * kCS + r16;
      const lds_f32* c7 = cb + (j7 < 32 ? j7 : 31) * kCS + r16;
      const lds_f32* c8 = cb + (j8 < 32 ? j8 : 31) * kCS + r16;
      const float ninf = -__builtin_inff();
      const float l0 = c1[0], l1 = c1[16], u0 = c7[32], u1 = c7[48], dg = c8[64];
      pix[e][0] = own[e][0];
      pix[e][1] = fmaxf(own[e][1], j1 < 32 ? l0 : ninf);
      pix[e][2] = fmaxf(own[e][2], j7 < 32 ? u0 : ninf);
      pix[e][3] = fmaxf(fmaxf(own[e][3], j1 < 32 ? l1 : ninf), fmaxf(j7 < 32 ? u1 : ninf, j8 < 32 ? dg : ninf));
      if (t >= a.P) continue;
      const int n = ps.n, tyy = ps.y, txx = ps.x;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int dy = d >> 1, dx = d & 1, py = 2 * tyy + dy, px = 2 * txx + dx;
        if (py >= a.Hp || px >= a.Wp) continue;  // a valid pixel's neighbour tiles are in its image
        pooled[(static_cast<size_t>(n * a.Hp + py) * a.Wp + px) * pc + fb + r16] = pix[e][d];
      }
    }
    // the upper part of straddling windows: pixels of tiles p0 - tx - 1 .. p0 - 1 (another workgroup's)
    // with a neighbour tile here; 3 pixels x 16 filters per tile
    const int back = a.tx + 1;
    const Pos pb = pos_of(p0 >= back ? p0 - back : 0);  // wave-uniform
    for (int it = lane; it < back * 3 * 16; it += 64) {
      const int f16 = it & 15, px3 = it >> 4, ob = px3 / 3, d = px3 - ob * 3 + 1;
      const int ot = p0 - back + ob;
      if (ot < 0) continue;
      // tile ot = pb + ob (p0 >= back here): ob <= tx, at most one row (and image) wrap
      int n = pb.n, tyy = pb.y, txx = pb.x + ob;
      if (txx >= a.tx) {
        txx -= a.tx;
        if (++tyy == a.ty) tyy = 0, ++n;
      }
      const int dy = d >> 1, dx = d & 1, py = 2 * tyy + dy, px = 2 * txx + dx;
      if (py >= a.Hp || px >= a.Wp) continue;
      const int lo = ot - p0;  // < 0: neighbour lo + j is here iff >= 0 (and < 32: j <= tx + 1 <= 32 + lo)
      float m = -__builtin_inff();
      bool any = false;
      if (dx && lo + 1 >= 0) m = fmaxf(m, cb[(lo + 1) * kCS + 16 * dy + f16]), any = true;
      if (dy && lo + a.tx >= 0) m = fmaxf(m, cb[(lo + a.tx) * kCS + 32 + 16 * dx + f16]), any = true;
      if (dy && dx && lo + a.tx + 1 >= 0) m = fmaxf(m, cb[(lo + a.tx + 1) * kCS + 64 + f16]), any = true;
      if (any) p2[(static_cast<size_t>(n * a.Hp + py) * a.Wp + px) * pc + fb + f16] = m;
    }
    return;
  }
  constexpr int kTS = 16;  // reads conflict-free in the b128 lane groups; writes 2-way, free for ds_write_b32
  constexpr int TW = 16 * G::NB;  // tiles per wave
  static_assert(G::kLdsBytes >= static_cast<size_t>(NW) * TW * kTS * 4, "epilogue scratch");
  float* tr = lds + wave * TW * kTS;
  const OutView o = a.out;
  int oy0[G::NB], ox0[G::NB], img[G::NB], trd[G::NB];
  const int grp = 4 * (lane & 3);
#pragma unroll
  for (int k = 0; k < G::NB; ++k) {
    const int t = (k * 64 + lane) >> 2, p = p0 + wm * TW + t;
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = p < a.P ? (pq % a.ty) * 4 : (1 << 28);  // out of range: never stored
    ox0[k] = tj * 4;
    img[k] = pq / a.ty;
    trd[k] = t * kTS + grp;
  }
#pragma unroll
  for (int q = 0; q < G::NQ; ++q) {
#pragma unroll
    for (int e = 0; e < G::NE; ++e) {
      float v = Y[q][e] + bv;
      if (a.relu) v = fmaxf(v, 0.f);
      tr[(16 * (e >> 2) + 4 * kg + (e & 3)) * kTS + r16] = v;
    }
    // same-wave LDS accesses complete in order: the reads see the writes above, and the next q's
    // writes cannot overtake these reads
#pragma unroll
    for (int k = 0; k < G::NB; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + trd[k]);
      const int oy = oy0[k] + q / 4, ox = ox0[k] + q % 4;
      if (oy < a.Ho && ox < a.Wo && (kStore || v4.x == -1.f))  // ABL 32: ReLU outputs are never -1
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(img[k] * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) *
                                               o.Cb + o.c_off + fb + grp) = v4;
    }
  }
}

}  // namespace anx::hip::wg16
