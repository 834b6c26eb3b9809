// Fused Winograd batched GEMM + output transform, fp32 on v_mfma_f32_32x32x2_f32 — the one kernel
// behind both Winograd convolutions (included by wino_gemm.hip and by the anx_wgemm A/B tool).
//
//   Conv2  F(3x3,5x5): NPT = 49 transform points, C = 96 channels, K = 256 filters
//   Conv1  polyphase F(3x3,3x3): NPT = 25 points, C = 48 polyphase channels, K = 96 filters
//
// A workgroup owns BM = 32*WM tiles x BN = 32*WN filters (one 32x32 MFMA tile per wave) and walks
// the NPT points: M_ab = V_ab[BM x C] . U_ab[C x BN] accumulates in one 16-register accumulator and
// is folded into the 3x3 outputs, Y[i][j] += A^T[i][a] A^T[j][b] M_ab, spread over the MFMAs of the
// NEXT point (two accumulators alternate). M never leaves registers; bias + ReLU + the NHWC store
// happen once at the end.
//
// Schedule (what differs from the round-2 kernels, winograd.hip / conv1_wino.hip history):
//  * K runs in slices of BK channels through an NST-slot LDS ring; slice it+NST-1 is issued right
//    after the barrier that opens slice it, so NST-2 slices of MFMAs cover a refill's latency (a
//    2-slot ring exposed ~15 % of the Conv2 GEMM as DMA wait: profiles/r03_wgemm_ab.md).
//  * The loop body covers UP points (UP*KS a multiple of NST), so every slice's ring slot, hence
//    every LDS read offset, is a compile-time immediate; the trip count is compile-time and the
//    last points are peeled with compile-time refill / wait counts.
//  * Each slice is its own scheduling region (sched_barrier on both sides of the wait + barrier):
//    the compiler had sunk a slice's last MFMAs below the next barrier, where the fold then waited
//    on their results.
//  * The fold of point ab-1 is spread over ALL slices of point ab (72 FMA pairs over KS*BK/2
//    MFMAs), pinned behind the MFMAs with sched_group_barrier, as scalar v_fma_f32 by default (a
//    packed FMA costs more than two scalar ones beside MFMAs: MI355X_MICROARCH.md, per-instruction
//    constants).
//  * One code path: buffer DMA only, no run-time probe or variant bits.
//
// Operand staging: buffer_load_dwordx4 ... lds (1 KiB per wave instruction; per-lane byte offsets in
// VGPRs once, the per-slice offset in an SGPR). LDS rows are BK floats unpadded; the 16-B unit u of
// row r is stored at u ^ swz(r), conflict-free for the ds_read_b128 fragment reads (checked per lane
// group for 4, 8 and 12 units per row); the swizzle is applied to the DMA's global source offsets.
//
// Reference op: convKernel (v3_cuda_only/src/layers_cuda.cu:20-46), one thread per output.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "anx/hip_sync.hpp"
#include "anx/ops.hpp"
#include "anx/winograd_f33.hpp"
#include "anx/winograd_f35.hpp"

namespace anx::hip::wg {

using f32x2 = __attribute__((ext_vector_type(2))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using lds_f32 = __attribute__((address_space(3))) float;
using lds_void = __attribute__((address_space(3))) void;

struct Args {
  const float* V;     // [P][NPT][vct]: this conv group's C channels start at V (vct >= C)
  const float* U;     // [NPT][u_rows][C]: row = filter, C floats
  const float* bias;  // [K]
  OutView out;        // conv output (NHWC through a view)
  int P, ty, tx, Ho, Wo;
  int n_ptiles, n_ntiles;  // set by the launcher from P and kg
  int kg;                  // filters of this launch (one conv group): n_ntiles = kg / BN
  int u_rows;          // filter rows per point in U (>= n_ntiles * BN)
  int vct;             // V floats per (tile, point): C, or groups * C
  int vbytes, ubytes;  // buffer sizes (< 2^31)
  int relu;
  float* p2;   // pool2 epilogue (gemm16_kernel<..., POOL>): straddling windows' partial maxima; out.base = pooled map
  int Hp, Wp;  // pooled map dims
};

// Fold coefficients per point, coef[ab][i*3 + j] = A^T[i][a] * A^T[j][b].
template <int NPT>
struct Coef {
  float v[NPT][9];
};
template <int NPT, int NN, class AT>
constexpr Coef<NPT> make_coef(const AT& at) {
  Coef<NPT> t{};
  for (int ab = 0; ab < NPT; ++ab)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) t.v[ab][i * 3 + j] = at[i][ab / NN] * at[j][ab % NN];
  return t;
}
static __constant__ Coef<49> c_coef49 = make_coef<49, 7>(anx::wino::kAT);
static __constant__ Coef<25> c_coef25 = make_coef<25, 5>(anx::wino33::kAT);

template <int NPT>
__device__ __forceinline__ const float* coef_row(int ab) {
  if constexpr (NPT == 49)
    return c_coef49.v[ab];
  else
    return c_coef25.v[ab];
}

constexpr int even_up(int ks, int nst) {  // smallest even UP with UP*ks % nst == 0
  int u = 2;
  while ((u * ks) % nst != 0) u += 2;
  return u;
}

// Compile-time shape of one configuration.
template <int NPT_, int C_, int WM_, int WN_, int BK_, int NST_>
struct Cfg {
  static constexpr int NPT = NPT_, C = C_, WM = WM_, WN = WN_, BK = BK_, NST = NST_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = 32 * WM, BN = 32 * WN, U4 = BK / 4;
  static constexpr int KS = C / BK, TOTAL = NPT * KS;              // K slices per point / in all
  static constexpr int A_INS = BM * U4 / 64, B_INS = BN * U4 / 64;  // 1-KiB DMA pieces per slice
  // piece q of an operand goes to wave q % NW: waves < INS % NW issue one more
  static constexpr int A_MAX = (A_INS + NW - 1) / NW, B_MAX = (B_INS + NW - 1) / NW;
  static constexpr int PW_MIN = A_INS / NW + B_INS / NW;  // the fewest pieces any wave issues per slice
  static constexpr int A_FL = BM * BK, STAGE = (BM + BN) * BK;  // floats
  static constexpr size_t kLdsBytes = static_cast<size_t>(NST) * STAGE * sizeof(float);
  static constexpr int UP = even_up(KS, NST);               // points per loop body
  static constexpr int NI = (TOTAL + 1 - NST) / (UP * KS);  // bodies whose refills all exist
  static constexpr int TAIL = NPT - NI * UP;                // peeled points
  static constexpr int MF = BK / 2;                         // MFMAs per slice
  static_assert(C % BK == 0 && A_INS * 64 == BM * U4 && B_INS * 64 == BN * U4, "tile shape");
  static_assert(U4 == 4 || U4 == 8 || U4 == 12, "swizzle defined for 4, 8, 12 units per row");
  static_assert(NST >= 2 && NI >= 1 && TAIL >= 1, "ring / loop shape");
};

template <int U4>
__device__ __forceinline__ int swz(int row) {
  if constexpr (U4 == 8)
    return (row >> 1) & 7;
  else
    return (row >> 2) & 3;
}

// compile-time loop: f(integral_constant<int, B>), ..., f(integral_constant<int, E - 1>)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm_lgkm() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
// ABL (A/B tool only; production instantiates 0): bit0 no fold, bit1 no DMA refills, bit2 no barrier,
// bit3 packed v_pk_fma_f32 fold instead of scalar, bit4 no sched_group_barrier pinning, bit5 no epilogue
// stores (the outputs are computed, never written).
template <class G, int ABL>
__global__ void __launch_bounds__(G::NT, 2) gemm_kernel(Args a) {
  constexpr int NPT = G::NPT, KS = G::KS, BK = G::BK, NW = G::NW, NST = G::NST, U4 = G::U4, MF = G::MF;
  constexpr bool kFold = !(ABL & 1), kDma = !(ABL & 2), kBar = !(ABL & 4), kPk = (ABL & 8) != 0, kPin = !(ABL & 16);
  constexpr bool kStore = !(ABL & 32);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: the DMA M0 values stay scalar
  const int wm = wave % G::WM, wn = wave / G::WM;
  // XCD-aware order: the n_ntiles workgroups that read one V slab get equal blockIdx.x % 8 (one XCD
  // under round-robin dispatch, so the slab comes from HBM/MALL once; speed only)
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nt = jb % a.n_ntiles, pt = (jb / a.n_ntiles) * 8 + xcd;
  if (pt >= a.n_ptiles) return;  // whole workgroup, before any DMA or barrier
  const int p0 = pt * G::BM, n0 = nt * G::BN;

  // per-lane byte offsets of this wave's DMA pieces (A piece q = wave + NW*i; B likewise)
  int voff[G::A_MAX], uoff[G::B_MAX];
#pragma unroll
  for (int i = 0; i < G::A_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::A_INS ? q : 0) * 64 + lane;
    const int row = U / U4, u = (U - row * U4) ^ swz<U4>(row);
    const int p = p0 + row;
    voff[i] = ((p < a.P ? p : 0) * NPT * a.vct + 4 * u) * 4;  // rows past P read tile 0, never stored
  }
#pragma unroll
  for (int i = 0; i < G::B_MAX; ++i) {
    const int q = wave + NW * i;
    const int U = (q < G::B_INS ? q : 0) * 64 + lane;
    const int row = U / U4, u = (U - row * U4) ^ swz<U4>(row);
    uoff[i] = ((n0 + row) * G::C + 4 * u) * 4;
  }
#if __HIP_DEVICE_COMPILE__  // the buffer-resource type exists in the device pass only
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.V), 0, a.vbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
#endif
  [[maybe_unused]] lds_f32* lds3 = (lds_f32*)(lds);
  // DMA of slice (ab, ks) into ring slot `slot`
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

  const int r = lane & 31, h = lane >> 5;
  // byte addresses (slot 0) of my A row's and B row's fragment units
  int ra[U4 / 2], rb[U4 / 2];
#pragma unroll
  for (int s4 = 0; s4 < U4 / 2; ++s4) {
    const int ua = 4 * ((h * (U4 / 2) + s4) ^ swz<U4>(wm * 32 + r));
    const int ub = 4 * ((h * (U4 / 2) + s4) ^ swz<U4>(wn * 32 + r));
    ra[s4] = ((wm * 32 + r) * BK + ua) * 4;
    rb[s4] = (G::A_FL + (wn * 32 + r) * BK + ub) * 4;
  }

  f32x2 Y[9][8];  // Y[q][e2]: output q of accumulator rows 2*e2, 2*e2+1
#pragma unroll
  for (int q = 0; q < 9; ++q)
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) Y[q][e2] = f32x2{0.f, 0.f};
  f32x16 acc[2] = {};
  float cq[2][9];  // fold coefficients of the point accumulated in acc[i], loaded as its MFMAs start

  auto frag = [&](int addr) { return *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(lds) + addr); };
  // fold pair J (0..71) of acc[FI] with cq[FI]: Y[q][e2] += c_q * (acc[2 e2], acc[2 e2 + 1])
  auto fold_pair = [&](auto J, auto FI) {
    constexpr int j = decltype(J)::value, fi = decltype(FI)::value, q = j >> 3, e2 = j & 7;
    if constexpr (kPk) {
      Y[q][e2] = __builtin_elementwise_fma(f32x2{cq[fi][q], cq[fi][q]}, f32x2{acc[fi][2 * e2], acc[fi][2 * e2 + 1]},
                                           Y[q][e2]);
    } else {
      Y[q][e2].x = __builtin_fmaf(cq[fi][q], acc[fi][2 * e2], Y[q][e2].x);
      Y[q][e2].y = __builtin_fmaf(cq[fi][q], acc[fi][2 * e2 + 1], Y[q][e2].y);
    }
  };

  // One K slice. LIT = the slice's position (compile-time) inside a UP-point body, or its absolute
  // index in the peeled prologue / tail (ABS = true); ab = its point (runtime in the loop). Every
  // schedule quantity is a compile-time constant: retire the slice (its DMA landed: vmcnt; everyone's:
  // barrier), refill the slot freed one slice ago with slice it+NST-1, then MF MFMAs into acc[ai] with
  // the next fragment group read ahead, and fold pairs [72*ks/KS, 72*(ks+1)/KS) of the previous point
  // (acc[ai^1]) spread behind them.
  auto slice = [&](int pb, auto LIT, auto ABS, auto FOLD) {
    constexpr int lit = decltype(LIT)::value;
    constexpr bool abs_it = decltype(ABS)::value, fold = decltype(FOLD)::value && kFold;
    constexpr int ks = lit % KS, ai = (lit / KS) & 1, slot = lit % NST, nlit = lit + NST - 1;
    // refills and in-flight counts: in the loop body every refill exists (NI bodies); peeled slices
    // know their absolute index
    constexpr bool refill = !abs_it || nlit < G::TOTAL;
    constexpr int ahead = abs_it ? ((G::TOTAL - 1 - lit) < NST - 2 ? (G::TOTAL - 1 - lit) : NST - 2) : NST - 2;
    const int ab = pb + lit / KS;
    __builtin_amdgcn_sched_barrier(0);
    // a wave that issues more pieces per slice waits a little early: safe
    constexpr int vm = kDma ? ahead * G::PW_MIN : 0;
    if constexpr (kBar)
      lds_barrier<vm>();
    else
      wait_vm_lgkm<vm>();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");  // keep the refill and the reads below the barrier
    if constexpr (refill) issue(pb + nlit / KS, nlit % KS, nlit % NST);
    if constexpr (ks == 0) {
      const float* cr = coef_row<NPT>(ab);
#pragma unroll
      for (int q = 0; q < 9; ++q) cq[ai][q] = cr[q];
    }
    constexpr int so = slot * G::STAGE * 4;
    constexpr int j0 = 72 * ks / KS, nj = 72 * (ks + 1) / KS - j0;
    f32x4 af[2], bf[2];
    af[0] = frag(ra[0] + so);
    bf[0] = frag(rb[0] + so);
    static_for<0, U4 / 2>([&](auto S4) {
      constexpr int s4 = decltype(S4)::value;
      if constexpr (s4 + 1 < U4 / 2) {
        af[(s4 + 1) & 1] = frag(ra[s4 + 1] + so);
        bf[(s4 + 1) & 1] = frag(rb[s4 + 1] + so);
      }
      static_for<0, 4>([&](auto S) {
        constexpr int sidx = decltype(S)::value, m = s4 * 4 + sidx;
        if constexpr (ks == 0 && m == 0)
          acc[ai] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[0][0], bf[0][0], f32x16{}, 0, 0, 0);
        else
          acc[ai] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s4 & 1][sidx], bf[s4 & 1][sidx], acc[ai], 0, 0, 0);
        if constexpr (fold)
          static_for<j0 + nj * m / MF, j0 + nj * (m + 1) / MF>(
              [&](auto J) { fold_pair(J, std::integral_constant<int, ai ^ 1>{}); });
      });
      if constexpr (kPin) {
        if constexpr (s4 + 1 < U4 / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // the next group's reads
        static_for<0, 4>([&](auto S) {
          constexpr int m = s4 * 4 + decltype(S)::value;
          constexpr int np = nj * (m + 1) / MF - nj * m / MF;  // fold pairs behind this MFMA
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
          if constexpr (fold && np > 0) __builtin_amdgcn_sched_group_barrier(0x002, kPk ? np : 2 * np, 0);
        });
      }
    });
    if constexpr (decltype(FOLD)::value && !kFold && ks == 0)
      Y[0][0] += f32x2{acc[ai ^ 1][0], acc[ai ^ 1][1]};  // probe: keep it live
  };
  using std::integral_constant;
  using T_ = integral_constant<bool, true>;
  using F_ = integral_constant<bool, false>;

  // prologue: slices 0 .. NST-2 in flight, then the first UP points (the first point folds nothing)
  static_for<0, NST - 1>([&](auto IT) {
    constexpr int it = decltype(IT)::value;
    issue(it / KS, it % KS, it);
  });
  static_for<0, G::UP * KS>([&](auto IT) {
    constexpr int it = decltype(IT)::value;
    slice(0, IT, T_{}, integral_constant<bool, (it >= KS)>{});
  });
  // steady state: UP points per trip (pb*KS is a multiple of NST: slots repeat per body)
  for (int pb = G::UP; pb < G::NI * G::UP; pb += G::UP) {
    static_for<0, G::UP * KS>([&](auto LIT) { slice(pb, LIT, F_{}, T_{}); });
  }
  // peeled tail: points NI*UP .. NPT-1 (refills stop, waits shrink)
  static_for<G::NI * G::UP * KS, G::TOTAL>([&](auto IT) { slice(0, IT, T_{}, T_{}); });
  // the last point's fold (not interleaved)
  static_for<0, 72>([&](auto J) { fold_pair(J, integral_constant<int, (NPT - 1) & 1>{}); });

  // Epilogue: bias + ReLU, then per output position q one LDS transpose of the wave's 32 tiles x 32
  // filters so each lane stores whole 16-B filter groups. D layout: lane (r, h) holds filter
  // n0 + wn*32 + r of tiles wm*32 + (e&3) + 8*(e>>2) + 4h.
  __syncthreads();  // the ring is idle (the last slice waited vmcnt(0)): reuse it as scratch
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
    oy0[k] = p < a.P ? (pq % a.ty) * 3 : (1 << 28);  // out of range: never stored
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
    // same-wave LDS accesses complete in order: the reads see the writes above, and the next q's
    // writes cannot overtake these reads
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(tr + ((k * 64 + lane) >> 3) * kTS + grp);
      const int oy = oy0[k] + q / 3, ox = ox0[k] + q % 3;
      if (oy < a.Ho && ox < a.Wo && (kStore || v4.x == -1.f))  // ABL 32: ReLU outputs are never -1
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(img[k] * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) *
                                               o.Cb + o.c_off + fb + grp) = v4;
    }
  }
}

}  // namespace anx::hip::wg
