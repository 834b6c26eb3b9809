// Implicit-GEMM convolution on CDNA4 f32 matrix cores (v_mfma_f32_32x32x2_f32).
//
// GEMM view: M = N*Ho*Wo output pixels (rows), N = filters (cols), K = F*F*Cg window taps.
//   A[m][k] = x[pixel_origin(m) + koff[k]]   (gathered on the fly from a pre-padded NHWC input)
//   B[k][n] = packed weight [n][k]            (KCFF repacked once, zero padded to the tile grid)
// The reference computes the same sums one output element per thread with no data reuse
// (convKernel, v3_cuda_only/src/layers_cuda.cu:20-46; v4_mpi_cuda/src/layers_mpi_cuda.cu:25-47).
//
// Design for gfx950:
//  * 256-thread workgroups = 4 wave64s; each wave owns a (TM*32) x (TN*32) accumulator tile in
//    TM*TN 16-register MFMA accumulators. f32-in MFMA runs at the f32 peak (157 TF), exact f32
//    (bitwise a k-ordered fmaf chain — MI355X_MICROARCH §Matrix cores).
//  * K is consumed in BK=32 tiles staged through ONE LDS array ([BM][BK+4] A, [BN][BK+4] B; the
//    +4-float pad makes the ds_read_b128 lane groups conflict-free: row stride 144 B).
//  * Inside a tile the k order is permuted so a lane's operands for 4 consecutive MFMA k-steps
//    are contiguous: lane half h at step s consumes k = h*BK/2 + s. A and B use the same
//    permutation, so D = A·B is unchanged; one ds_read_b128 feeds 4 MFMAs.
//  * Register-staged global prefetch of tile k+1 overlaps the MFMAs of tile k; 2-3 resident
//    workgroups per CU hide the two barriers per tile.
//  * Fused epilogue: + bias, optional ReLU, strided NHWC store through an OutView (can write
//    into the zero-bordered input of the next layer or into a channel slice of a concat).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "anx/ops.hpp"

namespace anx::hip {
namespace {

constexpr int kThreads = 256;
constexpr int kBK = 32;
constexpr int kLDA = kBK + 4;

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
// A gathers may start at any float (taps4 units of a C=3 image row): 4-byte alignment, still one
// global_load_dwordx4 (ROCm runs gfx9 in unaligned-access mode).
using f32x4u = __attribute__((ext_vector_type(4), aligned(4))) float;

struct ConvArgs {
  const float* x;
  const float* w;
  const int* koff;
  const float* bias;
  float* out;
  int M;          // N*Ho*Wo
  int HoWo, Wo;
  int Hp, Wp, C, S;
  int Cg, Kg;
  int kpad, kpad_n, ktiles;
  int Hb, Wb, Cb, h_off, w_off, c_off;
  int relu;
  int n_mtiles, n_ntiles;
};

template <int BM, int BN, int WAVES_M, int WAVES_N, bool VEC4, int NBUF>
__global__ void __launch_bounds__(kThreads, (BM * BN <= 128 * 96) ? 4 : 1) conv_mfma_kernel(ConvArgs a) {
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per workgroup");
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(TM * 32 == WM && TN * 32 == WN, "wave tile must be a multiple of 32");
  // A staging: VEC4 -> float4 chunks (BK/4 per row); scalar -> single floats (BK per row).
  constexpr int A_UNITS_PER_ROW = VEC4 ? kBK / 4 : kBK;
  constexpr int A_LOADS = BM * A_UNITS_PER_ROW / kThreads;
  static_assert(A_LOADS * kThreads == BM * A_UNITS_PER_ROW, "A tile must divide over 256 threads");
  constexpr int B_LOADS = BN * (kBK / 4) / kThreads;
  static_assert(B_LOADS * kThreads == BN * (kBK / 4), "B tile must divide over 256 threads");
  constexpr int A_ROW_STEP = kThreads / A_UNITS_PER_ROW;
  constexpr int B_ROW_STEP = kThreads / (kBK / 4);

  // One dynamic LDS array (guide §5 item 4a: a second __shared__ object can de-pipeline the
  // loop): [A tile | B tile | koff table]. The k->offset table is staged once per workgroup so
  // the per-tile gather never waits on a global load before issuing its A loads.
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kStage = (BM + BN) * kLDA;  // floats per LDS stage (A tile + B tile)
  float* As = lds;
  float* Bs = lds + BM * kLDA;
  int* koff_s = reinterpret_cast<int*>(lds + NBUF * kStage);
  // output pixel offset of each of the BM rows (-1 past M), filled by the prologue's divisions
  int* ooff_s = koff_s + a.kpad;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int g = blockIdx.z;

  // Tile coordinates: N-tiles of one M-tile are adjacent in launch order so they share the
  // gathered A rows through L2.
  const int bid = blockIdx.x;
  const int mt = bid / a.n_ntiles, nt = bid - mt * a.n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  const float* __restrict__ x = a.x + g * a.Cg;
  const float* __restrict__ wg = a.w + static_cast<size_t>(g) * a.kpad_n * a.kpad;
  for (int i = tid; i < a.kpad; i += kThreads) koff_s[i] = a.koff[i];

  // Per-thread A rows (fixed over the K loop): window origin offsets; rows past M point at
  // pixel 0 (always a valid address) and are zeroed by the a_ok mask after the load.
  const int a_unit = tid % A_UNITS_PER_ROW;
  int a_org[A_LOADS];
  unsigned a_ok = 0;
#pragma unroll
  for (int j = 0; j < A_LOADS; ++j) {
    const int row = tid / A_UNITS_PER_ROW + j * A_ROW_STEP;
    const int m = m0 + row;
    int oo = -1;
    a_org[j] = 0;
    if (m < a.M) {
      const int n = m / a.HoWo;
      const int rr = m - n * a.HoWo;
      const int oy = rr / a.Wo;
      const int ox = rr - oy * a.Wo;
      a_org[j] = ((n * a.Hp + oy * a.S) * a.Wp + ox * a.S) * a.C;
      oo = ((n * a.Hb + oy + a.h_off) * a.Wb + ox + a.w_off) * a.Cb + a.c_off;
    }
    if (tid % A_UNITS_PER_ROW == 0) ooff_s[row] = oo;
    a_ok |= (m < a.M ? 1u : 0u) << j;
  }
  __syncthreads();  // koff_s visible
  const int b_unit = tid % (kBK / 4);
  const float* b_src = wg + static_cast<size_t>(n0 + tid / (kBK / 4)) * a.kpad + b_unit * 4;

  using AReg = typename std::conditional<VEC4, f32x4, float>::type;
  AReg ra[A_LOADS];
  f32x4 rb[B_LOADS];
  bool kok = true;  // k chunk of the staged tile is real (not zero padding)

  // Unconditional loads from always-valid addresses; the zero-masking happens at LDS-store
  // time (store_tile), AFTER the MFMAs of the current tile, so no instruction consumes a loaded
  // value early and the loads stay in flight across the whole compute phase.
  auto load_tile = [&](int kt) {
    const int kbase = kt * kBK;
    const int ko_raw = koff_s[kbase + (VEC4 ? a_unit * 4 : a_unit)];
    kok = ko_raw >= 0;
    const int ko = kok ? ko_raw : 0;
#pragma unroll
    for (int j = 0; j < A_LOADS; ++j) {
      if constexpr (VEC4)
        ra[j] = *reinterpret_cast<const f32x4u*>(x + a_org[j] + ko);
      else
        ra[j] = x[a_org[j] + ko];
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j)
      rb[j] = *reinterpret_cast<const f32x4*>(b_src + static_cast<size_t>(j) * B_ROW_STEP * a.kpad + kbase);
  };
  auto store_tile = [&](int buf) {
    float* As_ = As + buf * kStage;
    float* Bs_ = Bs + buf * kStage;
#pragma unroll
    for (int j = 0; j < A_LOADS; ++j) {
      const int row = tid / A_UNITS_PER_ROW + j * A_ROW_STEP;
      const bool ok = kok && ((a_ok >> j) & 1u);
      if constexpr (VEC4)
        *reinterpret_cast<f32x4*>(As_ + row * kLDA + a_unit * 4) = ok ? ra[j] : f32x4{0.f, 0.f, 0.f, 0.f};
      else
        As_[row * kLDA + a_unit] = ok ? ra[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) {
      const int row = tid / (kBK / 4) + j * B_ROW_STEP;
      *reinterpret_cast<f32x4*>(Bs_ + row * kLDA + b_unit * 4) = rb[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int r = lane & 31, h = lane >> 5;
  const int a_rd = (wm * WM + r) * kLDA + h * (kBK / 2);
  const int b_rd = BM * kLDA + (wn * WN + r) * kLDA + h * (kBK / 2);

  auto compute = [&](const float* base) {
#pragma unroll
    for (int s4 = 0; s4 < kBK / 8; ++s4) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f32x4*>(base + a_rd + i * 32 * kLDA + s4 * 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f32x4*>(base + b_rd + j * 32 * kLDA + s4 * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();
  if constexpr (NBUF == 1) {
    // single LDS buffer: compute, barrier, restage, barrier
    for (int kt = 0; kt < a.ktiles; ++kt) {
      if (kt + 1 < a.ktiles) load_tile(kt + 1);
      compute(lds);
      __syncthreads();
      if (kt + 1 < a.ktiles) {
        store_tile(0);
        __syncthreads();
      }
    }
  } else {
    // two LDS buffers: the restage of tile k+1 goes to the buffer read in iteration k-1, which
    // every wave finished before the previous barrier -> one barrier per K tile.
    for (int kt = 0; kt < a.ktiles; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < a.ktiles) load_tile(kt + 1);
      compute(lds + cur * kStage);
      if (kt + 1 < a.ktiles) store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // Epilogue: D row (pixel) = (reg&3) + 8*(reg>>2) + 4*h ; D col (filter) = lane&31. The row ->
  // output offset map comes from LDS (4 consecutive rows per ds_read_b128), no divisions here.
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
      float* dst = a.out + g * a.Kg + f;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int o = oo[reg >> 2][reg & 3];
        if (o < 0) continue;
        float v = acc[i][j][reg] + bv;
        if (a.relu) v = fmaxf(v, 0.f);
        dst[o] = v;
      }
    }
  }
}

struct Variant {
  int BM, BN;
  bool vec4;
  int nbuf;
};
// id -> tile configuration (keep in sync with the dispatch switch in conv2d_mfma).
constexpr Variant kVariants[] = {
    {128, 128, true, 1},   // 0: large Cg%4==0 convs (conv2, conv3-5): 2x2 waves of 64x64
    {128, 96, false, 1},   // 1: conv1-like (C=3, K=96): 4x1 waves of 32x96, scalar gather
    {64, 64, true, 1},     // 2: small problems (batch 1): 2x2 waves of 32x32
    {64, 64, false, 1},    // 3: small problems, scalar gather
    {128, 128, false, 1},  // 4: large, scalar gather (Cg%4 != 0)
    {128, 128, true, 2},   // 5: = 0 with double-buffered LDS (one barrier per K tile)
    {128, 96, false, 2},   // 6: = 1 with double-buffered LDS
    {256, 128, true, 1},   // 7: 2x2 waves of 128x64 (8 accumulators per wave)
    {256, 96, false, 1},   // 8: conv1-like, 4x1 waves of 64x96 (6 accumulators per wave)
    {128, 96, true, 1},    // 9: conv1 with taps4 units: 4x1 waves of 32x96, 16-B gathers
    {256, 96, true, 1},    // 10: = 9 with 64x96 per wave
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
}  // namespace

bool conv_variant_valid(int kind, int id) {
  if (kind < 0 || kind > 1 || id < -1 || id >= kNumVariants) return false;
  return id < 0 || kVariants[id].vec4 == (kind == 0);
}

ConvPlan make_conv_plan(int N, int Hp, int Wp, int C, int K, int F, int S, int groups, int force_vec4,
                        int force_scalar) {
  if (!conv_variant_valid(0, force_vec4)) force_vec4 = -1;
  if (!conv_variant_valid(1, force_scalar)) force_scalar = -1;
  const int force[2] = {force_vec4, force_scalar};
  ConvPlan p{};
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
  p.vec4 = (p.Cg % 4 == 0 && C % 4 == 0) ? 1 : 0;
  // taps4 needs each filter row's (fw, c) floats contiguous (groups == 1); a forced scalar variant
  // (A/B tuning) keeps the scalar gather.
  p.taps4 = (!p.vec4 && groups == 1 && F * C >= 4 && force[1] < 0) ? 1 : 0;
  if (p.taps4) {
    p.kdim = F * 4 * ((F * C + 3) / 4);
    p.vec4 = 1;
  }
  p.kpad = (p.kdim + kBK - 1) / kBK * kBK;
  const long M = static_cast<long>(N) * p.Ho * p.Wo;
  const bool small = M * p.K < 256L * 128 * 128;  // fewer 128x128 tiles (all groups) than CUs
  if (p.Kg == 96 && !small)
    p.variant = p.vec4 ? 9 : 1;
  else if (small)
    p.variant = p.vec4 ? 2 : 3;
  else
    p.variant = p.vec4 ? 0 : 4;
  if (force[p.vec4 ? 0 : 1] >= 0) p.variant = force[p.vec4 ? 0 : 1];
  const int BN = kVariants[p.variant].BN;
  p.kpad_n = (p.Kg + BN - 1) / BN * BN;
  return p;
}

size_t packed_weight_floats(const ConvPlan& p) { return static_cast<size_t>(p.groups) * p.kpad_n * p.kpad; }
size_t koff_ints(const ConvPlan& p) { return static_cast<size_t>(p.kpad); }

void pack_conv_weights_host(const ConvPlan& p, const float* w_kcff, std::vector<float>& packed,
                            std::vector<int>& koff) {
  packed.assign(packed_weight_floats(p), 0.f);
  koff.assign(koff_ints(p), -1);
  if (p.taps4) {
    // filter row fh = L = F*C contiguous floats; unit u covers [start, start+4), the last unit
    // shifted back to [L-4, L): floats already covered by unit U-2 keep a zero weight there.
    const int L = p.F * p.C, U = (L + 3) / 4;
    for (int fh = 0; fh < p.F; ++fh)
      for (int u = 0; u < U; ++u)
        for (int e = 0; e < 4; ++e) {
          const int k = (fh * U + u) * 4 + e;
          const int start = u < U - 1 ? 4 * u : L - 4;
          const int f = start + e;
          koff[k] = fh * p.Wp * p.C + f;
          if (u == U - 1 && f < 4 * (U - 1)) continue;
          const int fw = f / p.C, c = f % p.C;
          for (int n = 0; n < p.Kg; ++n)
            packed[static_cast<size_t>(n) * p.kpad + k] = w_kcff[((static_cast<size_t>(n) * p.C + c) * p.F + fh) * p.F + fw];
        }
    return;
  }
  for (int g = 0; g < p.groups; ++g)
    for (int n = 0; n < p.Kg; ++n)
      for (int fh = 0; fh < p.F; ++fh)
        for (int fw = 0; fw < p.F; ++fw)
          for (int c = 0; c < p.Cg; ++c) {
            const int k = (fh * p.F + fw) * p.Cg + c;
            const int kf = g * p.Kg + n;
            packed[(static_cast<size_t>(g) * p.kpad_n + n) * p.kpad + k] =
                w_kcff[((static_cast<size_t>(kf) * p.Cg + c) * p.F + fh) * p.F + fw];
          }
  for (int fh = 0; fh < p.F; ++fh)
    for (int fw = 0; fw < p.F; ++fw)
      for (int c = 0; c < p.Cg; ++c) koff[(fh * p.F + fw) * p.Cg + c] = (fh * p.Wp + fw) * p.C + c;
}

hipError_t conv2d_mfma(const ConvPlan& p, const float* x, const float* wpacked, const int* koff,
                       const float* bias, OutView out, bool relu, hipStream_t s) {
  const long M = static_cast<long>(p.N) * p.Ho * p.Wo;
  if (M == 0) return hipSuccess;
  // 32-bit index math in the kernel: callers split larger batches (see Model::forward).
  if (static_cast<long>(p.N) * p.Hp * p.Wp * p.C >= (1L << 31) ||
      static_cast<long>(out.Hb) * out.Wb * out.Cb * p.N >= (1L << 31))
    return hipErrorInvalidValue;
  const Variant v = kVariants[p.variant];
  ConvArgs a{};
  a.x = x;
  a.w = wpacked;
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
  a.n_mtiles = static_cast<int>((M + v.BM - 1) / v.BM);
  a.n_ntiles = p.kpad_n / v.BN;
  dim3 grid(a.n_mtiles * a.n_ntiles, 1, p.groups);
  const size_t lds = static_cast<size_t>(v.nbuf) * (v.BM + v.BN) * kLDA * sizeof(float) +
                     static_cast<size_t>(p.kpad + v.BM) * sizeof(int);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (p.variant) {
    case 0: conv_mfma_kernel<128, 128, 2, 2, true, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 1: conv_mfma_kernel<128, 96, 4, 1, false, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 2: conv_mfma_kernel<64, 64, 2, 2, true, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 3: conv_mfma_kernel<64, 64, 2, 2, false, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 4: conv_mfma_kernel<128, 128, 2, 2, false, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 5: conv_mfma_kernel<128, 128, 2, 2, true, 2><<<grid, kThreads, lds, s>>>(a); break;
    case 6: conv_mfma_kernel<128, 96, 4, 1, false, 2><<<grid, kThreads, lds, s>>>(a); break;
    case 7: conv_mfma_kernel<256, 128, 2, 2, true, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 8: conv_mfma_kernel<256, 96, 4, 1, false, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 9: conv_mfma_kernel<128, 96, 4, 1, true, 1><<<grid, kThreads, lds, s>>>(a); break;
    case 10: conv_mfma_kernel<256, 96, 4, 1, true, 1><<<grid, kThreads, lds, s>>>(a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace anx::hip
