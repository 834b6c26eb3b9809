// Fused Winograd batched GEMM + output transform on the bf16 matrix cores with fp32-exact operands
// ("split bf16"; included by wino_gemm.hip and the anx_wgemm A/B tool).
//
// Every fp32 operand x is cut into three bf16 parts by truncation, x = h + m + l EXACTLY: h keeps the
// top 8 significant bits of x, r = x - h (exact) the remaining <= 16, m the top 8 of r and l = r - m
// (exact) the last <= 8, so l is itself a bf16 value. A bf16 x bf16 product is exact in fp32, so
//
//   NPROD = 9:  x*y = sum of all 9 part products, each exact; the MFMA sums them in fp32 — the
//               same arithmetic as an fp32 FMA dot product up to the order of the fp32 additions;
//   NPROD = 6:  drops m*l, l*m, l*l (each below 2^-21 |x*y|).
//
// v_mfma_f32_32x32x16_bf16 runs 16x the f32 MFMA rate (MI355X_MICROARCH.md, matrix cores), so 9
// products cost 9/16 of the v_mfma_f32_32x32x2_f32 time of the same GEMM and 6 cost 3/8.
//
// Operands: the transformed weights U are split once on the host into three bf16 planes
// Ub[point][plane][filter row][C]; V stays fp32 (the input transforms are unchanged) and each wave
// splits its A fragments in registers right after the LDS read (11 VALU per pair of values).
//
// Structure as wino_gemm.hpp (which see): 32x32 output tile per wave, BK = 48-channel K slices
// through an NST-slot LDS ring filled by buffer_load ... lds, the fold of point ab-1 into the 3x3
// outputs spread behind the MFMAs of point ab, two accumulators alternating, LDS-transposed 16-B
// NHWC stores. Per slice each wave runs 3 k-steps of 16 channels x NPROD MFMAs.
//
// LDS per ring slot: A = BM rows x 48 fp32 (12 16-B units per row, unit u of row r at u ^ ((r>>2)&3)),
// then B = 3 planes x BN rows x 48 bf16 (6 units per row, unit u at u ^ ((r>>3)&1)); both
// conflict-free for the ds_read_b128 fragment reads (4 lane groups of 16 lanes, one unit each).
//
// Reference op: convKernel (v3_cuda_only/src/layers_cuda.cu:20-46), one thread per output.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "wino_gemm.hpp"

namespace anx::hip::wsb {

using wg::Args;
using wg::coef_row;
using wg::f32x16;
using wg::f32x2;
using wg::f32x4;
using wg::lds_f32;
using wg::lds_void;
using wg::static_for;
using wg::wait_vm_lgkm;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

template <int NPT_, int C_, int WM_, int WN_, int NST_, int NPROD_, int MINB_ = 2>
struct Cfg {
  static constexpr int NPT = NPT_, C = C_, WM = WM_, WN = WN_, NST = NST_, NPROD = NPROD_, MINB = MINB_;
  static constexpr int BK = 48, KSTEP = BK / 16;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = 32 * WM, BN = 32 * WN;
  static constexpr int AU = BK / 4, BU = BK / 8;  // 16-B units per A row (fp32) / per B row-plane (bf16)
  static constexpr int KS = C / BK, TOTAL = NPT * KS;
  static constexpr int A_INS = BM * AU / 64, B_INS = 3 * BN * BU / 64;  // 1-KiB DMA pieces per slice
  static constexpr int A_MAX = (A_INS + NW - 1) / NW, B_MAX = (B_INS + NW - 1) / NW;
  static constexpr int PW_MIN = A_INS / NW + B_INS / NW;
  static constexpr int A_BYTES = BM * BK * 4, PLANE_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + 3 * PLANE_BYTES;
  static constexpr size_t kLdsBytes = static_cast<size_t>(NST) * STAGE_BYTES;
  static constexpr int UP = wg::even_up(KS, NST);
  static constexpr int NI = (TOTAL + 1 - NST) / (UP * KS);
  static constexpr int TAIL = NPT - NI * UP;
  static constexpr int MF = KSTEP * NPROD;  // MFMAs per slice
  static_assert(C % BK == 0 && A_INS * 64 == BM * AU && B_INS * 64 == 3 * BN * BU, "tile shape");
  static_assert(NST >= 2 && NI >= 1 && TAIL >= 1, "ring / loop shape");
  static_assert(NPROD == 9 || NPROD == 6, "part products");
};

__device__ __forceinline__ int swz_a(int row) { return (row >> 2) & 3; }
__device__ __forceinline__ int swz_b(int row) { return (row >> 3) & 1; }

__device__ __forceinline__ unsigned hi16x2(unsigned lo_src, unsigned hi_src) {
  // {upper half of lo_src, upper half of hi_src}: two bf16 truncations packed (v_perm_b32)
  return __builtin_amdgcn_perm(hi_src, lo_src, 0x07060302u);
}
__device__ __forceinline__ float hi_part(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }

// 8 fp32 values (k order j = 0..7) -> three packed bf16x8 parts, x = h + m + l exactly.
__device__ __forceinline__ void split8(const f32x4& x0, const f32x4& x1, bf16x8& h, bf16x8& m, bf16x8& l) {
  u32x4 H, M, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = i < 2 ? x0[2 * i] : x1[2 * i - 4], b = i < 2 ? x0[2 * i + 1] : x1[2 * i - 3];
    H[i] = hi16x2(__float_as_uint(a), __float_as_uint(b));
    const float ra = a - hi_part(a), rb = b - hi_part(b);
    M[i] = hi16x2(__float_as_uint(ra), __float_as_uint(rb));
    const float la = ra - hi_part(ra), lb = rb - hi_part(rb);
    L[i] = hi16x2(__float_as_uint(la), __float_as_uint(lb));
  }
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
  l = __builtin_bit_cast(bf16x8, L);
}

// Host/device-agnostic split of one fp32 value into its three bf16 parts (for the weight planes).
inline void split_host(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  auto bits = [](float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; };
  auto flt = [](uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; };
  const uint32_t xb = bits(x);
  h = static_cast<uint16_t>(xb >> 16);
  const float r = x - flt(xb & 0xffff0000u);
  const uint32_t rb = bits(r);
  m = static_cast<uint16_t>(rb >> 16);
  const float lo = r - flt(rb & 0xffff0000u);
  l = static_cast<uint16_t>(bits(lo) >> 16);
}

// ABL (A/B tool only; production instantiates 0): bit0 no fold, bit1 no DMA refills (times only).
template <class G, int ABL>
__global__ void __launch_bounds__(G::NT, G::MINB) sb_gemm_kernel(Args a) {
  constexpr int NPT = G::NPT, KS = G::KS, NW = G::NW, NST = G::NST;
  [[maybe_unused]] constexpr int BK = G::BK;  // device pass only
  constexpr bool kFold = !(ABL & 1), kDma = !(ABL & 2);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % G::WM, wn = wave / G::WM;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles, pt = (jb / a.n_ntiles) * 8 + xcd;
  if (pt >= a.n_ptiles) return;  // whole workgroup, before any DMA or barrier
  const int p0 = pt * G::BM, n0 = nt * G::BN;

  int voff[G::A_MAX], uoff[G::B_MAX];
#pragma unroll
  for (int i = 0; i < G::A_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::A_INS ? q : 0) * 64 + lane;
    const int row = U / G::AU, u = (U - row * G::AU) ^ swz_a(row);
    const int p = p0 + row;
    voff[i] = ((p < a.P ? p : 0) * NPT * a.vct + 4 * u) * 4;  // rows past P read tile 0, never stored
  }
#pragma unroll
  for (int i = 0; i < G::B_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::B_INS ? q : 0) * 64 + lane;
    const int plane = U / (G::BN * G::BU), rem = U - plane * (G::BN * G::BU);
    const int row = rem / G::BU, u = (rem - row * G::BU) ^ swz_b(row);
    uoff[i] = ((plane * a.u_rows + n0 + row) * G::C + 8 * u) * 2;
  }
#if __HIP_DEVICE_COMPILE__
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.V), 0, a.vbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
#endif
  [[maybe_unused]] lds_f32* lds3 = (lds_f32*)(lds);
  auto issue = [&](int ab, int ks, int slot) {
    if constexpr (kDma) {
#if __HIP_DEVICE_COMPILE__
      lds_f32* st = lds3 + slot * (G::STAGE_BYTES / 4);
      const int vso = (ab * a.vct + ks * BK) * 4;
      const int uso = (ab * 3 * a.u_rows * G::C + ks * BK) * 2;
#pragma unroll
      for (int i = 0; i < G::A_MAX; ++i)
        if ((G::A_INS % NW == 0) || wave + NW * i < G::A_INS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (lds_void*)(st + (wave + NW * i) * 256), 16, voff[i], vso, 0, 0);
#pragma unroll
      for (int i = 0; i < G::B_MAX; ++i)
        if ((G::B_INS % NW == 0) || wave + NW * i < G::B_INS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)(st + G::A_BYTES / 4 + (wave + NW * i) * 256), 16,
                                                   uoff[i], uso, 0, 0);
#endif
    }
  };

  const int r = lane & 31, h = lane >> 5;
  // byte addresses (slot 0) of this lane's fragment units: A k-step s: units 4s+2h, 4s+2h+1 of row
  // wm*32+r; B k-step s: unit 2s+h of row wn*32+r (plane 0; planes follow at PLANE_BYTES)
  int ra[2 * G::KSTEP], rb[G::KSTEP];
  {
    const int arow = wm * 32 + r, brow = wn * 32 + r;
#pragma unroll
    for (int s = 0; s < G::KSTEP; ++s) {
      ra[2 * s] = (arow * G::AU + ((4 * s + 2 * h) ^ swz_a(arow))) * 16;
      ra[2 * s + 1] = (arow * G::AU + ((4 * s + 2 * h + 1) ^ swz_a(arow))) * 16;
      rb[s] = G::A_BYTES + (brow * G::BU + ((2 * s + h) ^ swz_b(brow))) * 16;
    }
  }

  f32x2 Y[9][8];
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) Y[q][e2] = f32x2{0.f, 0.f};
  f32x16 acc[2] = {};
  float cq[2][9];

  auto frag4 = [&](int addr) { return *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(lds) + addr); };
  auto fragb = [&](int addr) { return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(lds) + addr); };
  auto fold_pair = [&](auto J, auto FI) {
    constexpr int j = decltype(J)::value, fi = decltype(FI)::value, q = j >> 3, e2 = j & 7;
    Y[q][e2].x = __builtin_fmaf(cq[fi][q], acc[fi][2 * e2], Y[q][e2].x);
    Y[q][e2].y = __builtin_fmaf(cq[fi][q], acc[fi][2 * e2 + 1], Y[q][e2].y);
  };

  auto slice = [&](int pb, auto LIT, auto ABS, auto FOLD) {
    constexpr int lit = decltype(LIT)::value;
    constexpr bool abs_it = decltype(ABS)::value, fold = decltype(FOLD)::value && kFold;
    constexpr int ks = lit % KS, ai = (lit / KS) & 1, slot = lit % NST, nlit = lit + NST - 1;
    constexpr bool refill = !abs_it || nlit < G::TOTAL;
    constexpr int ahead = abs_it ? ((G::TOTAL - 1 - lit) < NST - 2 ? (G::TOTAL - 1 - lit) : NST - 2) : NST - 2;
    const int ab = pb + lit / KS;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kDma)
      wait_vm_lgkm<ahead * G::PW_MIN>();
    else
      wait_vm_lgkm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if constexpr (refill) issue(pb + nlit / KS, nlit % KS, nlit % NST);
    if constexpr (ks == 0) {
      const float* cr = coef_row<NPT>(ab);
#pragma unroll
      for (int q = 0; q < 9; ++q) cq[ai][q] = cr[q];
    }
    constexpr int so = slot * G::STAGE_BYTES;
    constexpr int j0 = 72 * ks / KS, nj = 72 * (ks + 1) / KS - j0;
    static_for<0, G::KSTEP>([&](auto S) {
      constexpr int s = decltype(S)::value;
      const f32x4 x0 = frag4(ra[2 * s] + so), x1 = frag4(ra[2 * s + 1] + so);
      const bf16x8 bh = fragb(rb[s] + so), bm = fragb(rb[s] + so + G::PLANE_BYTES),
                   bl = fragb(rb[s] + so + 2 * G::PLANE_BYTES);
      bf16x8 ap[3], bp[3] = {bh, bm, bl};  // parts h, m, l
      split8(x0, x1, ap[0], ap[1], ap[2]);
      // part products (A part, B part), smallest first; NPROD = 6 starts at index 3
      constexpr int kPa[9] = {2, 2, 1, 2, 1, 0, 1, 0, 0}, kPb[9] = {2, 1, 2, 0, 1, 2, 0, 1, 0};
      static_for<9 - G::NPROD, 9>([&](auto I) {
        constexpr int i = decltype(I)::value;
        if constexpr (ks == 0 && s == 0 && i == 9 - G::NPROD)
          acc[ai] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[kPa[i]], bp[kPb[i]], f32x16{}, 0, 0, 0);
        else
          acc[ai] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[kPa[i]], bp[kPb[i]], acc[ai], 0, 0, 0);
      });
      if constexpr (fold)
        static_for<j0 + nj * s / G::KSTEP, j0 + nj * (s + 1) / G::KSTEP>(
            [&](auto J) { fold_pair(J, std::integral_constant<int, ai ^ 1>{}); });
    });
    if constexpr (decltype(FOLD)::value && !kFold && ks == 0) Y[0][0] += f32x2{acc[ai ^ 1][0], acc[ai ^ 1][1]};
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
  static_for<0, 72>([&](auto J) { fold_pair(J, integral_constant<int, (NPT - 1) & 1>{}); });

  // Epilogue (as wino_gemm.hpp): bias + ReLU, per output q an LDS transpose of the wave's 32 tiles x
  // 32 filters so each lane stores whole 16-B filter groups.
  __syncthreads();
  constexpr int kTS = 32 + 4;
  static_assert(G::kLdsBytes >= static_cast<size_t>(NW) * 32 * kTS * 4, "epilogue scratch");
  float* tr = lds + wave * 32 * kTS;
  const int fb = n0 + wn * 32;
  const float bv = a.bias ? a.bias[fb + r] : 0.f;
  const OutView o = a.out;
  int oy0[4], ox0[4], img[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + wm * 32 + ((k * 64 + lane) >> 3);
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = p < a.P ? (pq % a.ty) * 3 : (1 << 28);
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
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) >> 3) * kTS + grp);
      const int oy = oy0[k] + q / 3, ox = ox0[k] + q % 3;
      if (oy < a.Ho && ox < a.Wo)
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(img[k] * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) *
                                               o.Cb + o.c_off + fb + grp) = v4;
    }
  }
}

}  // namespace anx::hip::wsb
