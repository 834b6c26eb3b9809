// Fused Winograd batched GEMM + output transform for 4x4 output tiles, fp32 on v_mfma_f32_16x16x4_f32
// (included by wino_gemm.hip and the anx_wgemm A/B tool).
//
//   Conv2  F(4x4,5x5):            NN = 8 (64 transform points), C = 96 channels, K = 256 filters
//   Conv1  polyphase F(4x4,3x3):  NN = 6 (36 points),           C = 48 polyphase channels, K = 96
//
// Against the 3x3-tile kernel (wino_gemm.hpp) a 4x4 tile needs 64 / 16 = 4.0 multiplies per output
// instead of 49 / 9 = 5.4 (Conv2) and 36 / 16 = 2.25 instead of 25 / 9 = 2.8 (Conv1): ~21 % less
// matrix-core work and transform-domain traffic. 16 outputs per tile do not fit the 32x32 wave tile
// (16 x 16 fold registers), so a wave owns 16 tiles x 32 filters (two 16x16 MFMA blocks, 8 registers
// per output) and the output transform is applied separably along the point loop:
//
//   point (a, b):  Z[j] += A^T[j][b] M_ab      (b compile-time: zero coefficients cost nothing)
//   end of row a:  Y[i][j] += A^T[i][a] Z[j],  Z = 0
//
// 8 rows x (26 + 16) x 8 scalar FMAs per lane for Conv2 instead of 64 x 16 x 8. Each fold step rides
// in the MFMA stream of the next point (two accumulators alternate). The K slices stream through an
// NST-slot LDS ring fed by buffer_load ... lds, slots and read offsets compile-time per row body.
//
// Fragment layout (16x16x4): lane l holds A[tile l&15][k] / B[k][filter l&15] for the k of lane group
// g = l>>4; group g at MFMA step t (0..11 of a 48-channel slice) supplies k = 12g + t, so one
// ds_read_b128 per operand row feeds 4 steps. D: filter l&15, tile 4g + reg. The LDS rows rotate their
// 16-B units by 3*((row>>1)&3) (mod 12), conflict-free for this read pattern; the rotation is applied
// on the DMA's global source offsets.
//
// Reference op: convKernel (v3_cuda_only/src/layers_cuda.cu:20-46), one thread per output.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "anx/ops.hpp"
#include "anx/winograd_f43.hpp"
#include "anx/winograd_f45.hpp"
#include "wino_gemm.hpp"  // Args, static_for, wait_vm_lgkm

namespace anx::hip::wg16 {

using wg::Args;
using wg::f32x4;
using wg::lds_f32;
using wg::lds_void;
using wg::static_for;
using wg::wait_vm_lgkm;

// A^T of the two point sets, and its rows as compile-time functions of the point index
template <int NN>
struct AT {
  static constexpr float v(int i, int b) { return NN == 8 ? anx::wino45::kAT[i][b] : anx::wino43::kAT[i][b]; }
};
static __constant__ float c_at8[4][8] = {
    {1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 0.0f},
    {0.0f, 1.0f, -1.0f, 2.0f, -2.0f, 0.5f, -0.5f, 0.0f},
    {0.0f, 1.0f, 1.0f, 4.0f, 4.0f, 0.25f, 0.25f, 0.0f},
    {0.0f, 1.0f, -1.0f, 8.0f, -8.0f, 0.125f, -0.125f, 1.0f}};
static __constant__ float c_at6[4][6] = {{1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 0.0f},
                                         {0.0f, 1.0f, -1.0f, 0.5f, -2.0f, 0.0f},
                                         {0.0f, 1.0f, 1.0f, 0.25f, 4.0f, 0.0f},
                                         {0.0f, 1.0f, -1.0f, 0.125f, -8.0f, 1.0f}};

// NB: 16-filter MFMA blocks per wave (1: 16 tiles x 16 filters, ~110 registers, 4 waves per SIMD;
// 2: 16 x 32, ~250 registers, 2 waves per SIMD)
template <int NN_, int C_, int WM_, int WN_, int BK_, int NST_, int NB_, int MINB_ = 2>
struct Cfg {
  static constexpr int NN = NN_, NPT = NN * NN, C = C_, WM = WM_, WN = WN_, BK = BK_, NST = NST_, NB = NB_;
  static constexpr int MINB = MINB_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = 16 * WM, WB = 16 * NB, BN = WB * WN, U4 = BK / 4;
  static constexpr int KS = C / BK, TOTAL = NPT * KS, ROW = NN * KS;  // slices per point / in all / per row
  static constexpr int A_INS = BM * U4 / 64, B_INS = BN * U4 / 64;
  static constexpr int A_MAX = (A_INS + NW - 1) / NW, B_MAX = (B_INS + NW - 1) / NW;
  static constexpr int PW_MIN = A_INS / NW + B_INS / NW;
  static constexpr int A_FL = BM * BK, STAGE = (BM + BN) * BK;
  static constexpr size_t kLdsBytes = static_cast<size_t>(NST) * STAGE * sizeof(float);
  static constexpr int SG = U4 / 3;  // ds_read_b128 groups per slice (4 MFMA steps each)
  static_assert(U4 == 12, "the unit rotation is defined for 48-channel slices");
  static_assert(C % BK == 0 && A_INS * 64 == BM * U4 && B_INS * 64 == BN * U4, "tile shape");
  static_assert(ROW % NST == 0 && NN % 2 == 0 && NST >= 2, "ring / row shape");
};

__device__ __forceinline__ int rot(int row) { return 3 * ((row >> 1) & 3); }

template <class G, int ABL>
__global__ void __launch_bounds__(G::NT, G::MINB) gemm16_kernel(Args a) {
  constexpr int NN = G::NN, KS = G::KS, BK = G::BK, NW = G::NW, NST = G::NST, U4 = G::U4, NB = G::NB;
  constexpr bool kFold = !(ABL & 1), kDma = !(ABL & 2), kStore = !(ABL & 32);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % G::WM, wn = wave / G::WM;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles, pt = (jb / a.n_ntiles) * 8 + xcd;
  if (pt >= a.n_ptiles) return;  // whole workgroup, before any DMA or barrier
  const int p0 = pt * G::BM, n0 = nt * G::BN;

  // per-lane byte offsets of this wave's DMA pieces: slot su of row `row` holds logical unit
  // (su - rot(row)) mod 12
  int voff[G::A_MAX], uoff[G::B_MAX];
#pragma unroll
  for (int i = 0; i < G::A_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::A_INS ? q : 0) * 64 + lane;
    const int row = U / U4, u = (U - row * U4 + U4 - rot(row)) % U4;
    const int p = p0 + row;
    voff[i] = ((p < a.P ? p : 0) * G::NPT * a.vct + 4 * u) * 4;
  }
#pragma unroll
  for (int i = 0; i < G::B_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::B_INS ? q : 0) * 64 + lane;
    const int row = U / U4, u = (U - row * U4 + U4 - rot(row)) % U4;
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

  const int r16 = lane & 15, g = lane >> 4;
  // A rows wm*16 + r16 and B rows wn*32 + cb*16 + r16 share the rotation: group s4 of a slice reads
  // unit (3g + s4 + rot) mod 12 of each row. Byte addresses are formed per read (a few scalar-free
  // VALU ops) instead of held in 9 registers.
  const int ub = 3 * g + rot(r16);  // 0..20
  const int ra0 = (wm * 16 + r16) * BK * 4, rb00 = (G::A_FL + (wn * G::WB + r16) * BK) * 4;
  auto unit = [&](auto S4) {
    constexpr int s4 = decltype(S4)::value;
    const int u = ub + s4;
    return 16 * (u >= U4 ? u - U4 : u);
  };
  auto frag = [&](int addr) { return *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(lds) + addr); };

  f32x4 Y[16][NB];  // [i*4 + j][filter block]
  f32x4 Z[4][NB];   // row partials [j][block]
#pragma unroll
  for (int q = 0; q < 16; ++q)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) Y[q][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) Z[j][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc[2][NB] = {};  // [point parity][filter block]

  // fold of point b (compile-time) held in acc[pi]: Z[j] += A^T[j][b] acc
  auto zfold = [&](auto B, auto PI) {
    constexpr int b = decltype(B)::value, pi = decltype(PI)::value;
    static_for<0, 4>([&](auto J) {
      constexpr int j = decltype(J)::value;
      constexpr float c = AT<NN>::v(j, b);
      if constexpr (c != 0.f) {
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) Z[j][cb] = __builtin_elementwise_fma(f32x4{c, c, c, c}, acc[pi][cb], Z[j][cb]);
      }
    });
  };
  // end of row `ar` (runtime): Y[i][j] += A^T[i][ar] Z[j], Z = 0
  auto yfold = [&](int ar) {
    float ci[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ci[i] = NN == 8 ? c_at8[i][ar] : c_at6[i][ar];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int cb = 0; cb < NB; ++cb)
          Y[i * 4 + j][cb] = __builtin_elementwise_fma(f32x4{ci[i], ci[i], ci[i], ci[i]}, Z[j][cb], Y[i * 4 + j][cb]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) Z[j][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // One K slice: LIT = its index inside the row body (compile-time), ar = the row (runtime), LAST =
  // the peeled last row (refills stop at TOTAL). The first slice of point b > 0 carries the fold of
  // point b-1; the first slice of a row (b = 0) carries the previous row's last fold and its row fold.
  auto slice = [&](int ar, auto LIT, auto LAST) {
    constexpr int lit = decltype(LIT)::value;
    constexpr bool last = decltype(LAST)::value;
    constexpr int b = lit / KS, ks = lit % KS, pi = b & 1, slot = lit % NST;
    // slices issued after this one that may still be in flight (fewer in the last row's tail)
    constexpr int ahead = last ? ((G::ROW - 1 - lit) < NST - 2 ? (G::ROW - 1 - lit) : NST - 2) : NST - 2;
    __builtin_amdgcn_sched_barrier(0);
    wait_vm_lgkm<ahead * G::PW_MIN>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    {  // refill: slice lit + NST - 1 of this row body, or of the next row
      constexpr int nl = lit + NST - 1;
      if constexpr (!last || nl < G::ROW) {
        constexpr int nb = nl % G::ROW / KS, nks = nl % KS;
        issue((ar + nl / G::ROW) * NN + nb, nks, nl % NST);
      }
    }
    constexpr int so = slot * G::STAGE * 4;
    static_for<0, G::SG>([&](auto S4) {
      constexpr int s4 = decltype(S4)::value;
      const int un = unit(S4) + so;
      const f32x4 af = frag(ra0 + un);
      f32x4 bf[NB];
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) bf[cb] = frag(rb00 + cb * 16 * BK * 4 + un);
      static_for<0, 4>([&](auto S) {
        constexpr int s = decltype(S)::value;
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
          if constexpr (ks == 0 && s4 == 0 && s == 0)
            acc[pi][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[0], bf[cb][0], f32x4{}, 0, 0, 0);
          else
            acc[pi][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf[cb][s], acc[pi][cb], 0, 0, 0);
        }
        if constexpr (kFold && ks == 0 && s4 == 0 && s == 1) {  // behind the first MFMAs of the slice
          if constexpr (b > 0) {
            zfold(std::integral_constant<int, b - 1>{}, std::integral_constant<int, pi ^ 1>{});
          } else if (ar > 0) {  // uniform: the previous row's last point and row fold
            zfold(std::integral_constant<int, NN - 1>{}, std::integral_constant<int, 1>{});
            yfold(ar - 1);
          }
        }
      });
    });
  };
  using std::integral_constant;
  using T_ = integral_constant<bool, true>;
  using F_ = integral_constant<bool, false>;

  static_for<0, NST - 1>([&](auto IT) {
    constexpr int it = decltype(IT)::value;
    issue(it / KS, it % KS, it);
  });
  for (int ar = 0; ar < NN - 1; ++ar) static_for<0, G::ROW>([&](auto LIT) { slice(ar, LIT, F_{}); });
  static_for<0, G::ROW>([&](auto LIT) { slice(NN - 1, LIT, T_{}); });
  if constexpr (kFold) {
    zfold(integral_constant<int, NN - 1>{}, integral_constant<int, 1>{});
    yfold(NN - 1);
  } else {
    Y[0][0] += acc[1][0] + acc[0][0] + Z[0][0];  // probe: keep the accumulators live
  }
  static_assert(NB == 1 || NB == 2, "filter blocks per wave");

  // Epilogue: bias + ReLU, per output q an LDS transpose of the wave's 16 tiles x WB filters so each
  // lane stores whole 16-B filter groups. D: lane (r16, g) holds filter cb*16 + r16 of tile 4g + reg.
  __syncthreads();  // the ring is idle (every slice waited vmcnt(0)): reuse it as scratch
  constexpr int WB = G::WB, kTS = WB + 4, LPT = WB / 4, KT = 16 * LPT / 64;  // lanes per tile row, rows per pass
  static_assert(G::kLdsBytes >= static_cast<size_t>(NW) * 16 * kTS * 4, "epilogue scratch");
  float* tr = lds + wave * 16 * kTS;
  const int fb = n0 + wn * WB;
  float bv[NB];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) bv[cb] = a.bias ? a.bias[fb + cb * 16 + r16] : 0.f;
  const OutView o = a.out;
  int oy0[KT], ox0[KT], img[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int p = p0 + wm * 16 + (k * 64 + lane) / LPT;
    const int tj = p % a.tx, pq = p / a.tx;
    oy0[k] = p < a.P ? (pq % a.ty) * 4 : (1 << 28);  // out of range: never stored
    ox0[k] = tj * 4;
    img[k] = pq / a.ty;
  }
  const int grp = 4 * (lane % LPT);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = Y[q][cb][e] + bv[cb];
        if (a.relu) v = fmaxf(v, 0.f);
        tr[(4 * g + e) * kTS + cb * 16 + r16] = v;
      }
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) / LPT) * kTS + grp);
      const int oy = oy0[k] + q / 4, ox = ox0[k] + q % 4;
      if (oy < a.Ho && ox < a.Wo && (kStore || v4.x == -1.f))
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(img[k] * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) *
                                               o.Cb + o.c_off + fb + grp) = v4;
    }
  }
}

}  // namespace anx::hip::wg16
