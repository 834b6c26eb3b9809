// Launchers of the fused Winograd GEMM (wino_gemm.hpp) for Conv2 (F(3x3,5x5)) and Conv1 (polyphase
// F(3x3,3x3)). The production build instantiates one configuration per channel count; the anx_wgemm
// A/B tool (ANX_WGEMM_ABLATIONS) also instantiates the alternative ring / tile shapes and ablations.
//
// Measured at 300 images, each kernel alone (profiles/r03_wgemm_ab.md): 64x64 tiles, BK 48 and a 2-slot
// ring beat BK 32 x 4 slots and BK 16 x 6 slots (the deeper rings raised MFMA-busy but the chip then
// held a lower clock); Conv2 623 us (old fused kernel 649, bit-identical output), Conv1 380 us.
#include "wino_gemm.hpp"

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
#ifdef ANX_WGEMM_ABLATIONS
using C2_32x4 = wg::Cfg<49, 96, 2, 2, 32, 4>;    // 64 KiB ring: 2 slices in flight behind the current one
// 64 tiles x 128 filters, 8 waves, 72 KiB ring: a quarter less operand traffic per FLOP, but 636 vs 623 us
// alone at 300 images and 246-247 k vs 255 k images/s in the bench step (profiles/r03_conv2_wide_*)
using C2_64x128 = wg::Cfg<49, 96, 2, 4, 48, 2>;
using C2_64x64s3 = wg::Cfg<49, 96, 2, 2, 48, 3>;  // 64 x 64, 3-slot ring (72 KiB: still 2 workgroups per CU)
using C2_64x128s3 = wg::Cfg<49, 96, 2, 4, 48, 3>; // 64 x 128, 8 waves, 3-slot ring (108 KiB)
using C2_128x64 = wg::Cfg<49, 96, 4, 2, 48, 2>;   // 128 tiles x 64 filters, 8 waves (V read by 4 workgroups, U by half as many)
using C1_64x96 = wg::Cfg<25, 48, 2, 3, 48, 2>;   // 64 x 96 (every filter: V read once), 6 waves, 60 KiB ring
using C1_32x96 = wg::Cfg<25, 48, 1, 3, 48, 2>;   // 32 x 96, 3 waves, 48 KiB ring
using C1_48x2w4 = wg::Cfg<25, 48, 4, 1, 48, 2>;  // 128 x 32, 4 waves, 60 KiB ring, 2 per CU
#endif

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
#ifdef ANX_WGEMM_ABLATIONS
        case 1: e = launch_abl<C2_32x4>(a, s, occ, abl); break;
        case 2: e = launch_abl<C2_64x128>(a, s, occ, abl); break;
        case 3: e = launch_abl<C2_64x64s3>(a, s, occ, abl); break;
        case 4: e = launch_abl<C2_64x128s3>(a, s, occ, abl); break;
        case 5: e = launch_abl<C2_128x64>(a, s, occ, abl); break;
#endif
        default: break;
      }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
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
#ifdef ANX_WGEMM_ABLATIONS
    case 1: return launch_abl<C1_64x96>(a, s, occ, abl);
    case 2: return launch_abl<C1_32x96>(a, s, occ, abl);
    case 3: return launch_abl<C1_48x2w4>(a, s, occ, abl);
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace anx::hip

// ---- split-bf16 GEMMs (wino_gemm_sb.hpp): A/B build only. Measured slower than or level with the f32
// MFMA kernels (profiles/r03_sb_wgemm_ab.jsonl: Conv2 at 300 images x9 673 us, x6 580 us vs f32 627 us;
// Conv1 x9 431 / x6 378 vs 382): the per-wave A split costs 44 VALU per 16-channel k-step, more issue
// time than the 9 (or 6) bf16 MFMAs it feeds, and at 16x the MFMA rate the 64x64 tile (bounded by the
// 144 fold registers per wave) needs ~3x the L2->LDS bandwidth of the f32 kernel.
#ifdef ANX_WGEMM_ABLATIONS
#include "wino_gemm_sb.hpp"
namespace anx::hip {
namespace {

template <class G, int ABL>
hipError_t launch_sb(const wg::Args& a0, hipStream_t s, int occ) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(wsb::sb_gemm_kernel<G, ABL>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  wg::Args a = a0;
  a.n_ptiles = (a.P + G::BM - 1) / G::BM;
  a.n_ntiles = a.kg / G::BN;
  if (a.kg % G::BN || a.n_ntiles < 1 || a.u_rows < a.n_ntiles * G::BN) return hipErrorInvalidValue;
  const dim3 grid((a.n_ptiles + 7) / 8 * 8 * a.n_ntiles);
  wsb::sb_gemm_kernel<G, ABL><<<grid, G::NT, occupancy_lds(G::kLdsBytes, occ), s>>>(a);
  return hipGetLastError();
}

// <points, channels, waves along tiles, waves along filters, ring slots, part products>
using SB2x9 = wsb::Cfg<49, 96, 2, 2, 2, 9>;   // Conv2: 64 tiles x 64 filters, 60 KiB ring, 2 workgroups per CU
using SB2x6 = wsb::Cfg<49, 96, 2, 2, 2, 6>;
using SB2gx9 = wsb::Cfg<49, 48, 2, 2, 2, 9>;  // Conv2, 2 groups
using SB2gx6 = wsb::Cfg<49, 48, 2, 2, 2, 6>;
using SB1x9 = wsb::Cfg<25, 48, 2, 1, 2, 9>;   // Conv1: 64 tiles x 32 filters, 42 KiB ring
using SB1x6 = wsb::Cfg<25, 48, 2, 1, 2, 6>;

template <class G9, class G6>
hipError_t launch_sb_prod(const wg::Args& a, hipStream_t s, int occ, int nprod, int abl) {
  switch (nprod * 100 + abl) {
    case 900: return launch_sb<G9, 0>(a, s, occ);
    case 600: return launch_sb<G6, 0>(a, s, occ);
    case 901: return launch_sb<G9, 1>(a, s, occ);
    case 903: return launch_sb<G9, 3>(a, s, occ);
    case 601: return launch_sb<G6, 1>(a, s, occ);
    case 603: return launch_sb<G6, 3>(a, s, occ);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

void wino_split_planes_host(const std::vector<float>& u, int npt, int rows, int cols, std::vector<uint16_t>& ub) {
  ub.assign(static_cast<size_t>(npt) * 3 * rows * cols, 0);
  for (int ab = 0; ab < npt; ++ab)
    for (int n = 0; n < rows; ++n)
      for (int c = 0; c < cols; ++c) {
        uint16_t h, m, l;
        wsb::split_host(u[(static_cast<size_t>(ab) * rows + n) * cols + c], h, m, l);
        const size_t o = (static_cast<size_t>(ab) * 3 * rows + n) * cols + c, ps = static_cast<size_t>(rows) * cols;
        ub[o] = h;
        ub[o + ps] = m;
        ub[o + 2 * ps] = l;
      }
}

hipError_t wino_sb_gemm_conv2(const float* V, const uint16_t* Ub, const float* bias, OutView out, int P, int ty, int tx,
                              int Ho, int Wo, int C, int K, int groups, bool relu, hipStream_t s, int nprod, int occ,
                              int abl) {
  if (groups < 1 || C % groups || K % groups) return hipErrorInvalidValue;
  const int Cg = C / groups, Kg = K / groups;
  const long vb = static_cast<long>(P) * 49 * C * 4, ub = static_cast<long>(49) * 3 * K * Cg * 2;
  if ((Cg != 96 && Cg != 48) || Kg % 64 || vb >= (1L << 31) || ub >= (1L << 31) || out.Cb % 4 || out.c_off % 4)
    return hipErrorInvalidValue;
  if (P == 0) return hipSuccess;
  for (int g = 0; g < groups; ++g) {
    wg::Args a{};
    a.V = V + g * Cg;
    a.U = reinterpret_cast<const float*>(Ub + static_cast<size_t>(g) * Kg * Cg);  // bf16 planes (byte offsets)
    a.bias = bias ? bias + g * Kg : nullptr;
    a.out = out;
    a.out.c_off += g * Kg;
    a.P = P;
    a.ty = ty;
    a.tx = tx;
    a.Ho = Ho;
    a.Wo = Wo;
    a.kg = Kg;
    a.u_rows = K;
    a.vct = C;
    a.vbytes = static_cast<int>(vb - g * Cg * 4);
    a.ubytes = static_cast<int>(ub - static_cast<long>(g) * Kg * Cg * 2);
    a.relu = relu ? 1 : 0;
    const hipError_t e = Cg == 48 ? launch_sb_prod<SB2gx9, SB2gx6>(a, s, occ, nprod, abl)
                                  : launch_sb_prod<SB2x9, SB2x6>(a, s, occ, nprod, abl);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t wino_sb_gemm_conv1(const float* V, const uint16_t* Ub, const float* bias, OutView out, int P, int ty, int tx,
                              int Ho, int Wo, int K, bool relu, hipStream_t s, int nprod, int occ, int abl) {
  const long vb = static_cast<long>(P) * 25 * 48 * 4, ub = static_cast<long>(25) * 3 * K * 48 * 2;
  if (vb >= (1L << 31) || ub >= (1L << 31) || out.Cb % 4 || out.c_off % 4) return hipErrorInvalidValue;
  if (P == 0) return hipSuccess;
  wg::Args a{};
  a.V = V;
  a.U = reinterpret_cast<const float*>(Ub);
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
  return launch_sb_prod<SB1x9, SB1x6>(a, s, occ, nprod, abl);
}

}  // namespace anx::hip
#endif  // ANX_WGEMM_ABLATIONS
