// Launchers of the fused Winograd GEMMs: Conv2 on F(4x4,5x5) (wino_gemm16.hpp, the default since round 5)
// or F(3x3,5x5) (wino_gemm.hpp: grouped Conv2 and the conv2_tile=3 arm), and the two-kernel Conv1's
// polyphase F(3x3,3x3) GEMM (wino_gemm.hpp). The production build instantiates one configuration per
// shape; the anx_wgemm A/B tool (ANX_WGEMM_ABLATIONS) also instantiates a few alternatives and the cost
// probes of the production F(4,5) kernel.
//
// F(3x3,5x5), measured at 300 images alone (profiles/r03_wgemm_ab.md): 64x64 tiles, BK 48 and a 2-slot
// ring beat BK 32 x 4 slots and BK 16 x 6 slots (the deeper rings raised MFMA-busy but the chip then
// held a lower clock); Conv2 623 us (old fused kernel 649, bit-identical output), Conv1 380 us.
#include <type_traits>

#include "wino_gemm.hpp"
#include "wino_gemm16.hpp"

namespace anx::hip {
namespace {

int device_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

template <class G, int ABL>
hipError_t launch(const wg::Args& a0, hipStream_t s, int occ) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(wg::gemm_kernel<G, ABL>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  wg::Args a = a0;
  a.n_ptiles = (a.P + G::BM - 1) / G::BM;
  a.n_ntiles = a.kg / G::BN;
  if (a.kg % G::BN || a.n_ntiles < 1 || a.u_rows < a.n_ntiles * G::BN) return hipErrorInvalidValue;
  // auto cap: a launch with no more workgroups than CUs runs one per CU, so the workgroups of a
  // concurrent stream lane (and its transform kernels) find room on every CU (64 images per GPU as
  // 2 lanes: 218-219 k vs 209-211 k images/s, profiles/r03_occ_bench_ab.jsonl)
  if (occ < 0) occ = a.n_ptiles * a.n_ntiles <= device_cus() ? 1 : 0;
  const dim3 grid((a.n_ptiles + 7) / 8 * 8 * a.n_ntiles);
  wg::gemm_kernel<G, ABL><<<grid, G::NT, occupancy_lds(G::kLdsBytes, occ), s>>>(a);
  return hipGetLastError();
}

// Configurations: <points, channels, waves along tiles, waves along filters, K slice, ring slots>
using C2 = wg::Cfg<49, 96, 2, 2, 48, 2>;    // Conv2: 64 tiles x 64 filters, 48 KiB ring, 2 workgroups per CU
using C2g = wg::Cfg<49, 48, 2, 2, 48, 2>;   // Conv2 with 2 groups (48 channels per group)
using C1 = wg::Cfg<25, 48, 2, 1, 48, 2>;    // Conv1: 64 tiles x 32 filters, 2 waves, 4 workgroups per CU
// Round 3-4 alternatives (BK 32 x 4 slots, 64x128, 3-slot rings, 128x64; Conv1 64x96, 32x96, 128x32) were
// measured slower and removed from the A/B build: profiles/r03_wgemm_ab.md, profiles/r04_wgemm_ab/.

// The F(4x4,5x5) kernel (wino_gemm16.hpp): same Args, its own tile shape
template <class G, int ABL, bool POOL = false>
hipError_t launch16(const wg::Args& a0, hipStream_t s, int occ) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(wg16::gemm16_kernel<G, ABL, POOL>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  wg::Args a = a0;
  a.n_ptiles = (a.P + G::BM - 1) / G::BM;
  a.n_ntiles = a.kg / G::BN;
  if (a.kg % G::BN || a.n_ntiles < 1 || a.u_rows < a.n_ntiles * G::BN) return hipErrorInvalidValue;
  if (occ < 0) occ = a.n_ptiles * a.n_ntiles <= device_cus() ? 1 : 0;
  const dim3 grid((a.n_ptiles + 7) / 8 * 8 * a.n_ntiles);
  wg16::gemm16_kernel<G, ABL, POOL><<<grid, G::NT, occupancy_lds(G::kLdsBytes, occ), s>>>(a);
  return hipGetLastError();
}
// <waves along tiles, waves along filters, K slice, ring slots>: 32 tiles x 16 filters per wave
// 32 tiles x 64 filters, 4 waves, one point (all 96 channels) per K slice, 72 KiB ring: V read by 4 filter
// blocks instead of 8, one barrier and one refill wait per point (128 images alone: 273.2 us vs 291.8 with
// 48-channel slices, 298.0 for the F(3x3,5x5) kernel; profiles/r05_f45/wg45k_128.log)
using F45 = wg16::Cfg<1, 4, 96, 2>;
// The production schedule of F45 (knob conv2_sched = 1): the hand-scheduled slice (ABL bit 64) with the fold
// as one v_pk_fma_f32 burst at the slice start (fold mode 2 = 256, packed = 512) and the refill DMA issued by
// the compiler. 128 images alone: 255-260 vs 272-277 us, bitwise identical; the fold behind every MFMA ran
// 318 us, per group 287 / 263 (scalar / packed), the DMA moved into the statement 260-264
// (profiles/r06_conv2_sched/).
constexpr int kConv2Sched = kConv2SchedAbl;
static_assert(kConv2Sched == 64 + 256 + 512, "fold burst, packed, DMA by the compiler");
#ifdef ANX_WGEMM_ABLATIONS
// measured alone at 128 images (profiles/r05_f45/wg45_128_v2.log, wg45k_128.log): 64 x 64 on 8 waves
// 323 us, 128 x 32 317, 3-slot rings 303-315, 32 x 128 302: not kept as configurations
using F45_b48 = wg16::Cfg<1, 4, 48, 2>;      // the first production shape: 48-channel slices, 2 per point
using F45_k96x32 = wg16::Cfg<2, 2, 96, 2>;   // 64 x 32, one point per slice (275.8 us)
using F45_b48x32 = wg16::Cfg<2, 2, 48, 2>;   // 64 x 32, 48-channel slices
using F45_n1 = wg16::Cfg<2, 4, 96, 2, 1>;    // 32 x 64 on 8 waves of 16 x 16 (one MFMA block each: Y 64 registers,
                                             // 4 waves per SIMD instead of 2)
// Also measured at 128 / 64 images and not kept (profiles/r05_f45/wg45r*.log; within 1-2 %, the box
// noise): 48-channel slices x 4 slots, 32 x 6 slots, a separable output fold (T over an a-row's 8
// points, then Y once per row: 42 instead of 128 FMAs per point), filter blocks spread by XCD so each
// L2 holds a quarter of U.
#endif
template <class G>
hipError_t launch16_abl(const wg::Args& a, hipStream_t s, int occ, int abl) {
  if (abl == 0) return launch16<G, 0>(a, s, occ);
  if constexpr (std::is_same_v<G, F45>)
    if (abl == kConv2Sched) return launch16<G, kConv2Sched>(a, s, occ);  // hand-scheduled slice (knob conv2_sched)
#ifdef ANX_WGEMM_ABLATIONS
  if constexpr (std::is_same_v<G, F45>) {  // cost probes of the production shape only (compile time)
    if (abl == 64) return launch16<G, 64>(a, s, occ);
    if (abl == 65) return launch16<G, 65>(a, s, occ);
    if (abl == 67) return launch16<G, 67>(a, s, occ);
    // fold placement / packing / DMA placement of the hand-scheduled slice: 64 + 128 * fold mode + 512 * packed
    // + 1024 * DMA mode (wino_gemm16_sched.inc)
    if (abl == 704) return launch16<G, 704>(a, s, occ);
    if (abl == 1856) return launch16<G, 1856>(a, s, occ);
    if (abl == 2880) return launch16<G, 2880>(a, s, occ);
    if (abl == 3904) return launch16<G, 3904>(a, s, occ);
    if (abl == 2752) return launch16<G, 2752>(a, s, occ);
    if (abl == 1) return launch16<G, 1>(a, s, occ);
    if (abl == 2) return launch16<G, 2>(a, s, occ);
    if (abl == 3) return launch16<G, 3>(a, s, occ);
    if (abl == 4) return launch16<G, 4>(a, s, occ);
    if (abl == 16) return launch16<G, 16>(a, s, occ);
    if (abl == 32) return launch16<G, 32>(a, s, occ);
  }
#endif
  return hipErrorInvalidValue;
}

template <class G>
hipError_t launch_abl(const wg::Args& a, hipStream_t s, int occ, int abl) {
  switch (abl) {
    case 0: return launch<G, 0>(a, s, occ);
#ifdef ANX_WGEMM_ABLATIONS
    case 3: return launch<G, 3>(a, s, occ);
    case 32: return launch<G, 32>(a, s, occ);
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t wino_gemm_conv2(const float* V, const float* U, const float* bias, OutView out, int P, int ty, int tx, int Ho,
                           int Wo, int C, int K, int groups, bool relu, hipStream_t s, int occ, int abl, int cfg) {
  if (groups < 1 || C % groups || K % groups) return hipErrorInvalidValue;
  const int Cg = C / groups, Kg = K / groups;
  const long vb = static_cast<long>(P) * 49 * C * 4, ub = static_cast<long>(49) * K * Cg * 4;
  if ((Cg != 96 && Cg != 48) || Kg % 64 || vb >= (1L << 31) || ub >= (1L << 31) || out.Cb % 4 || out.c_off % 4)
    return hipErrorInvalidValue;
  if (P == 0) return hipSuccess;
  for (int g = 0; g < groups; ++g) {
    wg::Args a{};
    a.V = V + g * Cg;
    a.U = U + static_cast<size_t>(g) * Kg * Cg;
    a.bias = bias ? bias + g * Kg : nullptr;
    a.out = out;
    a.out.c_off += g * Kg;
    a.P = P;
    a.ty = ty;
    a.tx = tx;
    a.Ho = Ho;
    a.Wo = Wo;
    a.kg = Kg;
    a.u_rows = K;  // rows (ab*groups + g)*Kg + k: a point's rows of every group
    a.vct = C;
    a.vbytes = static_cast<int>(vb - g * Cg * 4);
    a.ubytes = static_cast<int>(ub - static_cast<long>(g) * Kg * Cg * 4);
    a.relu = relu ? 1 : 0;
    hipError_t e = hipErrorInvalidValue;
    if (Cg == 48)
      e = cfg < 0 ? launch_abl<C2g>(a, s, occ, abl) : hipErrorInvalidValue;
    else
      switch (cfg < 0 ? 0 : cfg) {
        case 0: e = launch_abl<C2>(a, s, occ, abl); break;
        default: break;
      }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t wino_gemm_conv2_f45(const float* V, const float* U, const float* bias, OutView out, int P, int ty, int tx,
                               int Ho, int Wo, int K, bool relu, hipStream_t s, int occ, int abl, int cfg) {
  const long vb = static_cast<long>(P) * 64 * 96 * 4, ub = static_cast<long>(64) * K * 96 * 4;
  if (K % 64 || vb >= (1L << 31) || ub >= (1L << 31) || out.Cb % 4 || out.c_off % 4) return hipErrorInvalidValue;
  if (P == 0) return hipSuccess;
  wg::Args a{};
  a.V = V;
  a.U = U;
  a.bias = bias;
  a.out = out;
  a.P = P;
  a.ty = ty;
  a.tx = tx;
  a.Ho = Ho;
  a.Wo = Wo;
  a.kg = K;
  a.u_rows = K;
  a.vct = 96;
  a.vbytes = static_cast<int>(vb);
  a.ubytes = static_cast<int>(ub);
  a.relu = relu ? 1 : 0;
  switch (cfg < 0 ? 0 : cfg) {
    case 0: return launch16_abl<F45>(a, s, occ, abl);
#ifdef ANX_WGEMM_ABLATIONS
    case 1: return launch16_abl<F45_b48>(a, s, occ, abl);
    case 2: return launch16_abl<F45_k96x32>(a, s, occ, abl);
    case 3: return launch16_abl<F45_b48x32>(a, s, occ, abl);
    case 4: return launch16_abl<F45_n1>(a, s, occ, abl);
#endif
    default: return hipErrorInvalidValue;
  }
}

hipError_t wino_gemm_conv2_f45_pool(const float* V, const float* U, const float* bias, float* pooled, float* p2, int P,
                                    int ty, int tx, int Ho, int Wo, int Hp, int Wp, int K, bool relu, hipStream_t s,
                                    int occ, bool sched) {
  const long vb = static_cast<long>(P) * 64 * 96 * 4, ub = static_cast<long>(64) * K * 96 * 4;
  // the epilogue's window walk: 4x4 tiles covering the map, a window's tiles within tx + 1 raster steps
  // of its first (< one workgroup's 32), pooled dims of a 3x3 / 2 pool
  if (K % 64 || vb >= (1L << 31) || ub >= (1L << 31) || ty * 4 < Ho || tx * 4 < Wo || tx + 1 > kConv2PoolTiles ||
      Hp != (Ho - 3) / 2 + 1 || Wp != (Wo - 3) / 2 + 1 || Ho < 3 || Wo < 3 || P % (ty * tx) ||
      static_cast<long>(P / (ty * tx)) * Hp * Wp * K >= (1L << 31))
    return hipErrorInvalidValue;
  if (P == 0) return hipSuccess;
  wg::Args a{};
  a.V = V;
  a.U = U;
  a.bias = bias;
  a.out = OutView{pooled, Hp, Wp, K, 0, 0, 0};
  a.P = P;
  a.ty = ty;
  a.tx = tx;
  a.Ho = Ho;
  a.Wo = Wo;
  a.kg = K;
  a.u_rows = K;
  a.vct = 96;
  a.vbytes = static_cast<int>(vb);
  a.ubytes = static_cast<int>(ub);
  a.relu = relu ? 1 : 0;
  a.p2 = p2;
  a.Hp = Hp;
  a.Wp = Wp;
  return sched ? launch16<F45, kConv2Sched, true>(a, s, occ) : launch16<F45, 0, true>(a, s, occ);
}

hipError_t wino_gemm_conv1(const float* V, const float* U, const float* bias, OutView out, int P, int ty, int tx, int Ho,
                           int Wo, int K, bool relu, hipStream_t s, int occ, int abl, int cfg) {
  const long vb = static_cast<long>(P) * 25 * 48 * 4, ub = static_cast<long>(25) * K * 48 * 4;
  if (vb >= (1L << 31) || ub >= (1L << 31) || out.Cb % 4 || out.c_off % 4) return hipErrorInvalidValue;
  if (P == 0) return hipSuccess;
  wg::Args a{};
  a.V = V;
  a.U = U;
  a.bias = bias;
  a.out = out;
  a.P = P;
  a.ty = ty;
  a.tx = tx;
  a.Ho = Ho;
  a.Wo = Wo;
  a.kg = K;
  a.u_rows = K;
  a.vct = 48;
  a.vbytes = static_cast<int>(vb);
  a.ubytes = static_cast<int>(ub);
  a.relu = relu ? 1 : 0;
  switch (cfg < 0 ? 0 : cfg) {
    case 0: return launch_abl<C1>(a, s, occ, abl);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace anx::hip

// The split-bf16 GEMMs (every fp32 operand as three exact bf16 parts on the bf16 matrix cores) were
// measured in round 3 and removed in round 5: slower than or level with these f32 MFMA kernels
// (profiles/r03_sb_wgemm_ab.jsonl; docs/ARCHITECTURE.md, Round-3 A/B results).
