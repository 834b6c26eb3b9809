// Conv1 as ONE kernel: polyphase Winograd F(3x3,3x3) with the input transform generated in LDS
// inside the GEMM (conv1_wino.hip explains the polyphase rewrite and the two-kernel form).
//
// The two-kernel form writes V [P][25][48] to HBM (1.73 MB per image, 2.8x the image) and the GEMM
// reads it back: 237 MB written + read per 128 images, ~29 % of the fp32 step's HBM traffic
// (profiles/r03_pmc_bytes_b128_after.md). Here a workgroup owns 64 tiles x ALL 96 filters, so each
// tile's V is built once, by the workgroup, from the image rows in L2:
//
//   a-step a (5 per workgroup): V_a[b][tile][ch] = sum_v B^T[b][v] t[v],
//                               t[v] = sum_u B^T[a][u] X'[tile][u][v][ch]   (same fmaf order as the
//                               band kernel, so V is bit-identical to the two-kernel form's)
//   point (a, b): M = V_ab[64 x 48] . U_ab[48 x 96] on v_mfma_f32_16x16x4_f32, folded into the 3x3
//                 outputs in registers: Y[i][j] += A^T[i][a] A^T[j][b] M.
//
// V_{a+1} is built (global loads of X' from L2 into registers, VALU) while the MFMAs of a-step a run
// and stored at its end; the two V buffers (5 points x 32 tiles x 48 ch, row stride 56 floats:
// conflict-free ds_read_b128 fragments) alternate by a-step. U_ab (18 KB per point) streams through a
// 3-slot LDS ring by buffer_load ... lds, one barrier per point (it also publishes V). Latency: U is
// issued two points ahead and each X' row one point before the point that consumes it, with every
// wait a compile-time vmcnt (the first form waited for everything at every point and ran the MFMA
// pipe ~29 % busy alone, 37 % of wave cycles in waits). 12 waves (3 per SIMD): wave (wm, wn) computes
// tiles 16 wm .. +15 x filters 16 wn .. +15 as one 16x16x4 MFMA block, so the fold keeps 36
// registers (9 outputs x 4 values) and three waves fit a SIMD with room for the V build. Bias + ReLU +
// the NHWC store through an LDS transpose (each 384-B output row of 96 filters written by 24 lanes,
// 16 B each).
//
// Reference op: convKernel (v3_cuda_only/src/layers_cuda.cu:20-46), one thread per output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <type_traits>
#include <utility>
#include <vector>

#include "anx/ops.hpp"
#include "anx/hip_sync.hpp"
#include "anx/winograd_f33.hpp"

namespace anx::hip {
namespace {

namespace w33 = anx::wino33;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using lds_f32 = __attribute__((address_space(3))) float;
using lds_void = __attribute__((address_space(3))) void;

[[maybe_unused]] constexpr int kPh = 4;
constexpr int kCh = 48, kN5 = 5, kPts = 25, kPitch = 12;
constexpr int kK = 96;                     // filters per workgroup (all of Conv1's)
constexpr int kTiles = 32;                 // tiles per workgroup
constexpr int kWaves = 12, kNT = 64 * kWaves;
constexpr int kVS = 56;                    // LDS row stride of V (floats): conflict-free b128 fragment reads
constexpr int kVBuf = kN5 * kTiles * kVS;  // floats per a-step V buffer
constexpr int kUSlot = kK * kCh;           // floats per U ring slot (one point)
constexpr int kUPieces = kUSlot / 256;     // 1-KiB DMA pieces per slot
constexpr int kUSlots = 3;                 // U ring slots: U_{p+2} is in flight while point p computes
constexpr int kOOB = 0x7ffffff0;           // a buffer offset past any extent: the load returns 0
constexpr int kOS = kK + 4;                // epilogue transpose row stride (floats)
constexpr int kDummy = 2 * kVBuf + kUSlots * kUSlot;  // 1-KiB scratch for the dummy DMAs
constexpr int kLdsFloats = kDummy + 256;
constexpr size_t kLds = kLdsFloats * sizeof(float);
static_assert(kLds <= 160 * 1024, "LDS");
// UPW (knob conv1_fused = 2): a private U ring per wave. Each wave DMAs the 16 filter rows its B fragments read
// (3 KiB per point, 3 pieces) into its own 2-slot ring, one point ahead, and waits for them with its own vmcnt:
// no other wave's DMA is read, so only the V publish at an a-step's first point needs a barrier (5 per
// workgroup instead of 25) and the waves drift between them. The two waves of a filter block load the same
// rows (2x the U traffic, L2 -> LDS).
constexpr int kUW = 16 * kCh;                                    // floats per wave per slot
constexpr int kLdsFloatsW = 2 * kVBuf + kWaves * 2 * kUW;       // 145,408 B
constexpr size_t kLdsW = kLdsFloatsW * sizeof(float);
static_assert(kLdsW <= 160 * 1024 && kUW == 3 * 256, "per-wave U ring: three 1-KiB pieces per point");
static_assert(kUSlot % 256 == 0 && kUPieces <= 2 * kWaves && kUPieces >= kWaves, "U ring pieces: 1 or 2 per wave");

// V_a takes X' row u iff B^T[a][u] != 0
constexpr bool needs_row(int av, int u) { return av < kN5 && w33::kBT[av][u] != 0.f; }
// Every X' row is loaded ONCE per thread and kept in registers while any later V needs it (round 4
// re-loaded it for every V_a that takes it: 16 row loads per thread instead of 5, ~710 MB of L2 -> VGPR
// traffic per 128 images; the no-load cost probe ran the kernel 37 us faster, profiles/r05_conv1_abl/).
// The rows V_0 takes (0-3) load in the prologue; a row first taken by a later V_a (row 4: V_4) loads
// four points before the point that adds it into t (point b = u of a-step a - 1).
constexpr bool prologue_row(int u) { return needs_row(0, u); }
constexpr int first_a(int u) {
  for (int a = 1; a < kN5; ++a)
    if (needs_row(a, u)) return a;
  return kN5;
}
constexpr int late_load_pt(int u) {
  return prologue_row(u) || first_a(u) >= kN5 ? -1 : ((first_a(u) - 1) * kN5 + u >= 4 ? (first_a(u) - 1) * kN5 + u - 4 : 0);
}
// the X' row loaded at point p (-1: none)
constexpr int loads_at(int p) {
  for (int u = 0; u < kN5; ++u)
    if (p >= 0 && late_load_pt(u) == p) return u;
  return -1;
}
constexpr int x_ops(int p) { return p >= 0 && loads_at(p) >= 0 ? kN5 : 0; }
static_assert(9 * kTiles * kOS <= kDummy, "epilogue scratch: nine position images below the dummy DMA slot");
// pool1 epilogue: candidate pooled pixels are those whose window starts in tiles p0 - kPoolBack .. p0 + 31
// (a window's tiles span at most tx + 1 raster indices: kPoolBack >= tx + 1, checked by the launcher)
constexpr int kPoolBack = 20, kPoolSlots = 4 * (kPoolBack + kTiles);
constexpr int kPoolList = 9 * kTiles * kOS;  // the slot list after the nine position images
// then per listed pixel 12 ints: its 9 window pixels' LDS float offsets (-1: another workgroup's),
// the destination's element offset, whether it goes to p1, padding (16-B aligned entries)
constexpr int kPoolEnt = 12, kPoolOffs = (kPoolList + 1 + kPoolSlots + 3) / 4 * 4;
// a row of 96 -inf after the table: a window pixel another workgroup owns reads it (no branch per read, so the
// nine reads of a pooled pixel issue back to back behind one wait)
constexpr int kPoolSent = kPoolOffs + kPoolSlots * kPoolEnt;
static_assert(kPoolSent % 4 == 0 && kPoolSent + kK <= kLdsFloats && kPoolSent + kK <= kLdsFloatsW, "pool sentinel row");
static_assert(kPoolOffs + kPoolSlots * kPoolEnt <= kLdsFloats && kPoolOffs + kPoolSlots * kPoolEnt <= kLdsFloatsW &&
                  kPoolSlots <= kNT, "pool1 slot list");
static_assert(kTiles * 24 == kNT, "V build: one (tile, channel pair) per thread");

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

// 16-B unit u of U row r sits at unit u ^ swz(r) of its LDS row (12 units per row): conflict-free
// ds_read_b128 of the B fragments (16 filter rows x 4 units per lane group; (r >> 2) & 3 left 2-way
// conflicts for this access pattern)
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 3; }

struct Conv1FusedArgs {
  const float* x;     // [N][Hin][W][3] image rows of the tile
  const float* U;     // [25][96][48] transformed filters
  const float* bias;  // [96]
  OutView out;
  int P, ty, tx, Ho, Wo, Hin, rowf;  // rowf = W * 3 floats per image row
  int xbytes, ubytes;                // buffer-resource extents (< 2^31)
  int n_ptiles, per_xcd;
  int relu;
  // POOL: pool1 (3x3 / 2 max) in the epilogue. Pooled pixels whose window lies in this workgroup's
  // 32 tiles are written to `out` (the conv2 input window); a window that straddles two workgroups'
  // tile ranges gets the partial max of each: the lower workgroup's into `out`, the upper's into p1
  // ([N][Hp][Wp][96]), merged by the consumer (pool1_straddles()).
  float* p1;
  int Hp, Wp;
  unsigned long long* dbg;  // ABL bit 64 (ANX_CONV1_PHASES diagnostics): per-workgroup stamps, else null
};

// UM: where U lives -- 0 the shared 3-slot LDS ring (every wave's DMA, a barrier per point), 1 a private
// 2-slot LDS ring per wave (own DMA, own vmcnt; barriers only at a-step starts), 2 registers (each wave loads
// its B fragments from L2 one point ahead; no U in LDS at all)
template <bool POOL, int ABL = 0, int UM = 0>
__global__ void __launch_bounds__(kNT, 3) conv1_fused_kernel(Conv1FusedArgs a) {
  // (two accumulation chains per point, odd k-steps on the second, measured slower with the per-wave ring:
  // main loop 48.5 k vs 44.2 k clk, profiles/r06_conv1_upw/)
  constexpr bool UPW = UM == 1, UREG = UM == 2;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: the DMA M0 values stay scalar
  const int wm = wave & 1, wn = wave >> 1;
  // consecutive tile blocks on one XCD (they read overlapping image rows: L2 reuse; speed only)
  const int pt = (blockIdx.x & 7) * a.per_xcd + (blockIdx.x >> 3);
  if (pt >= a.n_ptiles) return;  // whole workgroup, before any barrier
  const int p0 = pt * kTiles;
  // ABL bit 64: wave 0's s_memtime at the phase boundaries (diagnostic build only; stamps go to a.dbg)
  constexpr bool kStamp = (ABL & 64) != 0;
  unsigned long long stamp[7] = {}, rt0 = 0;
  if constexpr (kStamp) {
    stamp[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
#if __HIP_DEVICE_COMPILE__
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, a.ubytes, 0x00020000);
#endif
  lds_f32* lds3 = (lds_f32*)(lds);
  float* const vbuf = lds;                                   // [2][5][kTiles][kVS]
  [[maybe_unused]] lds_f32* const uring = lds3 + 2 * kVBuf;  // [kUSlots][kK][kCh], swizzled units

  // ---- U ring: point ab into slot ab % kUSlots, issued two points ahead (pieces q = wave, wave + 12)
  int uoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave + kWaves * i, U = (q < kUPieces ? q : 0) * 64 + lane;
    const int row = U / 12, u = (U - row * 12) ^ swz(row);
    uoff[i] = q < kUPieces ? (row * kCh + 4 * u) * 4 : kOOB;  // no second piece: the dummy reads zeros
  }
  // Every wave issues exactly 2 vector-memory ops per point, unconditionally: the waves without a
  // second 1-KiB piece DMA zeros (out-of-range source) into a 1-KiB scratch row instead, so the compiler's (and the schedule's)
  // vmcnt values count the same ops on every wave (with a conditional second piece the compiler
  // assumed none and its waits for the X' rows also waited for the U DMA just issued).
  // UPW: this wave's pieces: units i * 64 + lane of its 16 rows (filters 16 wn ..), swizzled as the shared ring
  [[maybe_unused]] int uoffw[3];
  [[maybe_unused]] lds_f32* const uringw = uring + wave * 2 * kUW;
  if constexpr (UPW) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int U = i * 64 + lane, row = U / 12, u = (U - row * 12) ^ swz(row);
      uoffw[i] = ((wn * 16 + row) * kCh + 4 * u) * 4;
    }
  }
  // UREG: this wave's B fragments of point ab, g = 0..2: filter row brow, channels 16 g + 4 h4 .. +3
  [[maybe_unused]] f32x4 ub[2][3];
  [[maybe_unused]] const int ubo = ((wn * 16 + (lane & 15)) * kCh + 4 * (lane >> 4)) * 4;
  auto issue_u = [&](auto AB) {
    [[maybe_unused]] constexpr int ab = decltype(AB)::value;
    if constexpr ((ABL & 2) != 0) return;
#if __HIP_DEVICE_COMPILE__
    if constexpr (UREG) {
#pragma unroll
      for (int g = 0; g < 3; ++g)
        ub[ab & 1][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ur, ubo + 64 * g, ab * kUSlot * 4, 0));
      return;
    }
    if constexpr (UPW) {
      lds_f32* st = uringw + (ab % 2) * kUW;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)(st + i * 256), 16, uoffw[i], ab * kUSlot * 4, 0, 0);
      return;
    }
    lds_f32* st = uring + (ab % kUSlots) * kUSlot;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)(st + wave * 256), 16, uoff[0], ab * kUSlot * 4, 0, 0);
    lds_f32* st2 = wave + kWaves < kUPieces ? st + (wave + kWaves) * 256 : lds3 + kDummy;  // scalar select
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_void*)st2, 16, uoff[1], ab * kUSlot * 4, 0, 0);
#endif
  };

  // ---- the V build slot of this thread: tile bt, channels 2 bc, 2 bc + 1 (phase row rh, floats 2 bc % 12
  // .. +1 of the 12-float (rw, c) run)
  const int bt = tid / 24, bc = tid - bt * 24, rh = (2 * bc) / 12, bf2 = 2 * bc - rh * 12;
  const int bp = p0 + bt;
  const bool bval = bp < a.P;
  int btj = 0, bti = 0, bn = 0;
  if (bval) {
    btj = bp % a.tx;
    const int pq = bp / a.tx;
    bti = pq % a.ty;
    bn = pq / a.ty;
  }
  const int row0 = bti * kPitch + rh;               // image row of u = 0 (this slot's phase row)
  const int col0 = btj * kPitch * 3 + bf2;          // float of v = 0 inside the row
  [[maybe_unused]] const int xoff = ((bn * a.Hin + row0) * a.rowf + col0) * 4;
  // X'[u][v] (2 channels): image row 12 ti + 4u + rh, floats (12 tj + 4v) * 3 + bf2 .. +1 (zero outside).
  // Every load is issued by every lane (a lane outside the image reads past the buffer's extent, which
  // returns 0), so each X' row is exactly kN5 vector-memory ops per wave and the schedule's vmcnt
  // values are compile-time. At the row's last float (o + 1 == rowf) the pair's .y is the next row's
  // first float (or, past the buffer, 0: the range check is per dword): t's .y for that column is
  // zeroed once per a-step before V is formed (vpart), instead of a select per load.
  bool rok[kN5], cpart[kN5];
  int offv[kN5];  // per column v: this lane's byte offset, or past the extent (zeros)
#pragma unroll
  for (int i = 0; i < kN5; ++i) {
    const int o = col0 + 12 * i;
    rok[i] = bval && row0 + kPh * i < a.Hin;
    offv[i] = o < a.rowf ? xoff : kOOB;
    cpart[i] = o + 1 == a.rowf;
  }
  auto load_x = [&](int u, int v) -> f32x2 {
    f32x2 d = {0.f, 0.f};
    if constexpr ((ABL & 1) != 0) return f32x2{static_cast<float>(offv[v] + u), static_cast<float>(v)};
#if __HIP_DEVICE_COMPILE__
    const int so = (kPh * u * a.rowf + 12 * v) * 4;
    d = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(xr, rok[u] ? offv[v] : kOOB, so, 0));
#endif
    return d;
  };
  f32x2 t[kN5];
  auto t_zero = [&]() {
#pragma unroll
    for (int v = 0; v < kN5; ++v) t[v] = f32x2{0.f, 0.f};
  };
  // t = B^T d over u, then V = t B over v: the fmaf expressions and order of conv1_wino_band_kernel
  auto t_add = [&](auto A, auto Uc, const f32x2 (&d)[kN5]) {
    constexpr int av = decltype(A)::value, u = decltype(Uc)::value;
    constexpr float c = w33::kBT[av][u];
    if constexpr (c != 0.f)
#pragma unroll
      for (int v = 0; v < kN5; ++v) {
        t[v].x = __builtin_fmaf(c, d[v].x, t[v].x);
        t[v].y = __builtin_fmaf(c, d[v].y, t[v].y);
      }
  };
  auto v_store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < kN5; ++v) t[v].y = cpart[v] ? 0.f : t[v].y;  // the row's last float has no pair
    float* vb = vbuf + buf * kVBuf + bt * kVS + 2 * bc;
    sfor<0, kN5>([&](auto Bc) {
      constexpr int b = decltype(Bc)::value;
      f32x2 s = {0.f, 0.f};
      sfor<0, kN5>([&](auto Vc) {
        constexpr int v = decltype(Vc)::value;
        constexpr float c = w33::kBT[b][v];
        if constexpr (c != 0.f) {
          s.x = __builtin_fmaf(c, t[v].x, s.x);
          s.y = __builtin_fmaf(c, t[v].y, s.y);
        }
      });
      *reinterpret_cast<f32x2*>(vb + b * kTiles * kVS) = s;
    });
  };

  // ---- MFMA fragments (v_mfma_f32_16x16x4_f32): A[row = lane & 15][k = lane >> 4], B[k = lane >> 4][col =
  // lane & 15]; k-step 4g + i uses channel 16g + 4(lane >> 4) + i (one ds_read_b128 per operand per g)
  const int r16 = lane & 15, h4 = lane >> 4;
  // the epilogue's bias, loaded here: issued at the epilogue it exposed a global-load latency per workgroup
  const float bv = a.bias ? a.bias[wn * 16 + r16] : 0.f;
  const int a_off = (wm * 16 + r16) * kVS + 4 * h4;
  const int brow = wn * 16 + r16;
  int b_off[3];  // UPW: row r16 of this wave's ring slot (swz(brow) == swz(r16): 16 wn leaves bits 1-2)
#pragma unroll
  for (int g = 0; g < 3; ++g) b_off[g] = (UPW ? r16 : brow) * kCh + 4 * ((4 * g + h4) ^ swz(brow));
  f32x4 Y[9];  // Y[q]: output q of the block's 4 accumulator rows
#pragma unroll
  for (int q = 0; q < 9; ++q) Y[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  // separable fold: T[j] = sum_b A^T[j][b] M_ab over the a-step's points, then Y[i][j] += A^T[i][a] T[j]
  // at its end (352 instead of 484 FMAs per wave and tile block)
  f32x4 T[3];

  // Schedule (points p = 5a + b in order). At point p a wave: waits for U_p (its own DMA: vmcnt; every
  // wave's: the barrier, which also publishes V_a), issues U_{p+2} (two points of MFMAs cover its
  // latency) and a late X' row if one loads at p, runs point p's MFMAs and fold, then adds X' row b
  // (resident) into t (V_{a+1}). V_{a+1} is stored at the end of a-step a. vmcnt is in order: the wait
  // at point p leaves in flight exactly the ops issued after U_p (inflight below).
  f32x2 xrow[kN5][kN5];  // X' rows of this thread's (tile, channel pair), each loaded once (see late_load_pt)
  // prologue: U_0, U_1 in flight; the rows V_0 takes loaded (kept), V_0 built and stored
  issue_u(std::integral_constant<int, 0>{});
  if constexpr (UM == 0) issue_u(std::integral_constant<int, 1>{});  // UPW / UREG: one point ahead (2 slots)
  // (the compiler issues U_0 after the X' row loads of V_0; pinning it ahead of them measured slower: the
  // rows are the prologue's critical path, 4.5 k -> 5.1 k clk, profiles/r06_conv1_upw/)
  t_zero();
  sfor<0, kN5>([&](auto Uc) {
    constexpr int u = decltype(Uc)::value;
    if constexpr (prologue_row(u))
#pragma unroll
      for (int v = 0; v < kN5; ++v) xrow[u][v] = load_x(u, v);
  });
  sfor<0, kN5>([&](auto Uc) {
    constexpr int u = decltype(Uc)::value;
    if constexpr (prologue_row(u)) t_add(std::integral_constant<int, 0>{}, Uc, xrow[u]);
  });
  v_store(0);
  t_zero();
  if constexpr (kStamp) stamp[1] = __builtin_amdgcn_s_memtime();

  sfor<0, kN5>([&](auto Ac) {
    constexpr int av = decltype(Ac)::value;
    const float* vb = vbuf + (av & 1) * kVBuf;
#pragma unroll
    for (int j = 0; j < 3; ++j) T[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    sfor<0, kN5>([&](auto Bc) {
      constexpr int b = decltype(Bc)::value, p = av * kN5 + b;
      // in flight past this barrier: the ops issued after U_p (at point p - 2: its X' row, if any; at
      // point p - 1: U_{p+1} and its X' row): this wave's U_p has landed, X' rows finish on their own
      constexpr int inflight = (p + 1 < kPts ? 2 : 0) + x_ops(p - 1) + x_ops(p - 2);
      // UPW: U_p was issued at point p - 1 (the prologue for p = 0); after it only point p - 1's X' row loads
      constexpr int inflight_w = x_ops(p - 1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (UREG) {
        if constexpr (b == 0) lds_barrier<-1>();  // V_a published; U is in registers (the compiler waits for it)
      } else if constexpr (UPW) {
        if constexpr (b == 0)
          lds_barrier<inflight_w>();  // V_a published (and every wave past a-step a - 1's reads of its buffer)
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(inflight_w) : "memory");  // this wave's own U_p pieces
      } else if constexpr ((ABL & 4) != 0)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(inflight) : "memory");
      else
        lds_barrier<inflight>();
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
      if constexpr (UPW || UREG) {
        // slot (p + 1) % 2 held U_{p-1}, read by this wave only, at point p - 1 (its MFMAs consumed the reads)
        if constexpr (p + 1 < kPts) issue_u(std::integral_constant<int, p + 1>{});
      } else if constexpr (p + 2 < kPts) {
        issue_u(std::integral_constant<int, p + 2>{});  // slot of point p - 1: free
      }
      if constexpr (loads_at(p) >= 0) {
        constexpr int r = loads_at(p);
#pragma unroll
        for (int v = 0; v < kN5; ++v) xrow[r][v] = load_x(r, v);
      }
      __builtin_amdgcn_sched_barrier(0);  // loads issued before the MFMAs
      const float* vp = vb + b * kTiles * kVS + a_off;
      const float* up = UPW ? reinterpret_cast<const float*>(lds + 2 * kVBuf + wave * 2 * kUW + (p % 2) * kUW)
                            : reinterpret_cast<const float*>(lds + 2 * kVBuf + (p % kUSlots) * kUSlot);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        const f32x4 af = *reinterpret_cast<const f32x4*>(vp + 16 * g);
        f32x4 bf;
        if constexpr (UREG)
          bf = ub[p & 1][g];
        else
          bf = *reinterpret_cast<const f32x4*>(up + b_off[g]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[i], acc, 0, 0, 0);
      }
      // fold, first half: T[j] += A^T[j][b] M_ab (compile-time coefficients; zero ones skipped)
      if constexpr ((ABL & 16) != 0) asm volatile("" ::"v"(acc));
      sfor<0, 3>([&](auto Jc) {
        constexpr int j = decltype(Jc)::value;
        constexpr float c = w33::kAT[j][b];
        if constexpr (c != 0.f && (ABL & 16) == 0)
#pragma unroll
          for (int i = 0; i < 4; ++i) T[j][i] = __builtin_fmaf(c, acc[i], T[j][i]);  // scalar v_fma_f32
      });
      // pinned here (the empty asm takes t and T as operands: the DAG scheduler had sunk the adds to the
      // a-step's end, where their in-order vmcnt also waited for the U DMA just issued)
      if constexpr (needs_row(av + 1, b) && (ABL & 8) != 0) {
#pragma unroll
        for (int v = 0; v < kN5; ++v) asm volatile("" ::"v"(xrow[b][v]));
      } else if constexpr (needs_row(av + 1, b)) {
        t_add(std::integral_constant<int, av + 1>{}, Bc, xrow[b]);
#pragma unroll
        for (int v = 0; v < kN5; ++v) asm volatile("" : "+v"(t[v]));
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) asm volatile("" : "+v"(T[j]));
      if constexpr (b == kN5 - 1) {  // fold, second half: Y[i][j] += A^T[i][a] T[j]
        sfor<0, 9>([&](auto Qc) {
          constexpr int q = decltype(Qc)::value;
          constexpr float c = w33::kAT[q / 3][av];
          if constexpr (c != 0.f)
#pragma unroll
            for (int i = 0; i < 4; ++i) Y[q][i] = __builtin_fmaf(c, T[q % 3][i], Y[q][i]);
        });
#pragma unroll
        for (int q = 0; q < 9; ++q) asm volatile("" : "+v"(Y[q]));
      }
      if constexpr (b == kN5 - 1 && av + 1 < kN5 && (ABL & 8) == 0) {
        // V_{a+1} into the other buffer (last read in a-step a - 1, before this a-step's first barrier);
        // published by the barrier of point (a + 1, 0)
        v_store((av + 1) & 1);
        t_zero();
      }
    });
  });

  if constexpr (kStamp) stamp[2] = __builtin_amdgcn_s_memtime();
  // ---- epilogue: per output position q, bias + ReLU into an LDS image [32 tiles][96 filters], then
  // 16-B row-contiguous stores. D layout: lane holds col = lane & 15 (filter), rows 4 (lane >> 4) + i.
  const int f = wn * 16 + r16;
  const OutView o = a.out;
  float* tr = lds;
  const int st = tid / (kK / 4), sq = tid - st * (kK / 4);  // this thread's store: tile st, filters 4 sq .. +3
  const int sp = p0 + st;
  int sn = 0, sti = 0, stj = 0;
  if (sp < a.P) {
    stj = sp % a.tx;
    const int pq = sp / a.tx;
    sti = pq % a.ty;
    sn = pq / a.ty;
  }
  if constexpr (POOL) {
    // pool1 from the same [9 positions][32 tiles][kOS] image. A pooled pixel (py, px) reads conv1 rows
    // 2py .. 2py+2 x cols 2px .. 2px+2: tiles (2py/3 .. (2py+2)/3) x (2px/3 .. (2px+2)/3), raster
    // indices gm .. gM with gM - gm <= tx + 1 < 32, so at most two workgroups' tile ranges meet in one
    // window. The workgroup owning gm writes its partial max to `out`, the one owning gM (if another)
    // to p1. Slots: the pooled pixels whose top-left tile is one of tiles p0 - 20 .. p0 + 31 (1-4 per
    // tile), compacted into a list in LDS, then 24 threads (4 filters each) per listed pixel.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's last fragment reads are done: the LDS is scratch now
    int* plist = reinterpret_cast<int*>(lds + kPoolList);  // [0] count, [1 ..] pixel descriptors
#pragma unroll
    for (int q = 0; q < 9; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = Y[q][i] + bv;
        if (a.relu) v = fmaxf(v, 0.f);
        tr[(q * kTiles + wm * 16 + 4 * h4 + i) * kOS + f] = v;
      }
    if (tid == 0) plist[0] = 0;
    if (tid < kK) lds[kPoolSent + tid] = -INFINITY;
    const int ipt = a.ty * a.tx;  // tiles per image
    int desc = -1;
    if (tid < kPoolSlots) {
      const int gt = p0 - kPoolBack + (tid >> 2), dyi = (tid >> 1) & 1, dxi = tid & 1;
      if (gt >= 0 && gt < a.P) {
        const int n = gt / ipt, r = gt - n * ipt, tyy = r / a.tx, txx = r - tyy * a.tx;
        // pooled rows whose window starts in tile row tyy: 2py in [3 tyy, 3 tyy + 2]
        const int py = ((3 * tyy + 1) >> 1) + dyi, px = ((3 * txx + 1) >> 1) + dxi;
        const bool ok = dyi < 2 - (tyy & 1) && dxi < 2 - (txx & 1) && py < a.Hp && px < a.Wp;
        if (ok) {
          const int gM = n * ipt + ((2 * py + 2) / 3) * a.tx + (2 * px + 2) / 3;
          if (gt >= p0)
            desc = ((n * 32 + py) * 32 + px) * 2;  // lower owner: `out`
          else if (gM >= p0)
            desc = ((n * 32 + py) * 32 + px) * 2 + 1;  // upper owner of a straddling window: p1
        }
      }
    }
    __syncthreads();  // position images and the zeroed count visible
    if constexpr (kStamp) stamp[3] = __builtin_amdgcn_s_memtime();
    if (desc >= 0) plist[1 + atomicAdd(&plist[0], 1)] = desc;
    __syncthreads();
    const int nlist = plist[0];
    // per listed pixel, once: the LDS offsets of its window pixels this workgroup owns, its destination
    using i32x4 = __attribute__((ext_vector_type(4))) int;
    int* ent = reinterpret_cast<int*>(lds + kPoolOffs);
    for (int k = tid; k < nlist; k += kNT) {
      const int d = plist[1 + k];
      const int up = d & 1, px = (d >> 1) & 31, py = (d >> 6) & 31, n = d >> 11;
      int e[kPoolEnt];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int y = 2 * py + i, tyy = y / 3, ry = y - 3 * tyy;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int x = 2 * px + j, txx = x / 3, rx = x - 3 * txx;
          const int lt = n * ipt + tyy * a.tx + txx - p0;
          e[i * 3 + j] = static_cast<unsigned>(lt) < static_cast<unsigned>(kTiles) ? ((ry * 3 + rx) * kTiles + lt) * kOS
                                                                                  : kPoolSent;
        }
      }
      e[9] = up ? ((n * a.Hp + py) * a.Wp + px) * kK : ((n * o.Hb + py + o.h_off) * o.Wb + px + o.w_off) * o.Cb + o.c_off;
      e[10] = up;
      e[11] = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        *reinterpret_cast<i32x4*>(ent + k * kPoolEnt + 4 * q) = i32x4{e[4 * q], e[4 * q + 1], e[4 * q + 2], e[4 * q + 3]};
    }
    __syncthreads();
    if constexpr (kStamp) stamp[4] = __builtin_amdgcn_s_memtime();
    for (int it = tid; it < ((ABL & 32) != 0 ? 0 : nlist) * (kK / 4); it += kNT) {
      const int k = it / (kK / 4), fq = it - k * (kK / 4);
      const i32x4 e0 = *reinterpret_cast<const i32x4*>(ent + k * kPoolEnt);
      const i32x4 e1 = *reinterpret_cast<const i32x4*>(ent + k * kPoolEnt + 4);
      const i32x4 e2 = *reinterpret_cast<const i32x4*>(ent + k * kPoolEnt + 8);
      const int off[9] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x};
      f32x4 v[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) v[i] = *reinterpret_cast<const f32x4*>(tr + off[i] + 4 * fq);
      f32x4 m = v[0];
#pragma unroll
      for (int i = 1; i < 9; ++i) m = f32x4{fmaxf(m.x, v[i].x), fmaxf(m.y, v[i].y), fmaxf(m.z, v[i].z), fmaxf(m.w, v[i].w)};
      float* dst = (e2.z ? a.p1 : o.base) + static_cast<size_t>(static_cast<unsigned>(e2.y)) + 4 * fq;
      *reinterpret_cast<f32x4*>(dst) = m;
    }
    if constexpr (kStamp) {
      stamp[5] = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pooled stores acknowledged
      stamp[6] = __builtin_amdgcn_s_memtime();
      if (tid == 0) {
        unsigned long long* d = a.dbg + static_cast<size_t>(pt) * 10;
#pragma unroll
        for (int i = 0; i < 7; ++i) d[i] = stamp[i];
        d[7] = rt0;
        d[8] = __builtin_amdgcn_s_memrealtime();
        // HW_ID (CU / SE of this wave) and XCC_ID: which CU ran this workgroup (the gap to the next one)
        d[9] = (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32) |
               static_cast<unsigned>(__builtin_amdgcn_s_getreg((31 << 11) | 4));
      }
    }
  } else {
    // all nine output positions' images at once (9 x 32 x 100 floats = 115 KB of the 128 KB): one
    // barrier and nine back-to-back stores per thread instead of a write / barrier / store / barrier
    // round per position. The images reach into the U ring's slots, so no DMA may still be landing.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's last fragment reads are done: the LDS is scratch now
#pragma unroll
    for (int q = 0; q < 9; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = Y[q][i] + bv;
        if (a.relu) v = fmaxf(v, 0.f);
        tr[(q * kTiles + wm * 16 + 4 * h4 + i) * kOS + f] = v;
      }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int oy = sti * 3 + q / 3, ox = stj * 3 + q % 3;
      if (sp < a.P && oy < a.Ho && ox < a.Wo)
        *reinterpret_cast<f32x4*>(o.base + (static_cast<size_t>(sn * o.Hb + oy + o.h_off) * o.Wb + ox + o.w_off) * o.Cb +
                                  o.c_off + 4 * sq) = *reinterpret_cast<const f32x4*>(tr + (q * kTiles + st) * kOS + 4 * sq);
    }
  }
}

}  // namespace

bool conv1_fused_eligible(const Conv1WinoPlan& w, const OutView& out) {
  return w.K == kK && w.W * 3 >= 4 && out.Cb % 4 == 0 && out.c_off % 4 == 0 &&
         static_cast<long>(w.N) * w.Hin * w.W * 3 * 4 < (1L << 31);
}

namespace {
// ANX_CONV1_PHASES: medians of wave 0's phase clocks per workgroup, and per CU the gap between one
// workgroup's end and the next one's start (s_memrealtime, 100 MHz)
void conv1_phase_report(const std::vector<unsigned long long>& h, int n) {
  auto median = [](std::vector<double> v) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const char* names[6] = {"prologue", "main loop", "epilogue: Y to LDS + barrier", "pool list + table",
                          "pooled max + store issue", "store drain"};
  std::vector<double> ph[6], life;
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> per_cu;
  for (int b = 0; b < n; ++b) {
    const unsigned long long* d = &h[static_cast<size_t>(b) * 10];
    if (d[0] == 0) continue;
    for (int i = 0; i < 6; ++i) ph[i].push_back(static_cast<double>(d[i + 1] - d[i]));
    life.push_back(static_cast<double>(d[8] - d[7]) * 10.0);  // ns
    const unsigned long long hw = d[9] & 0xffffffffull, cu = ((d[9] >> 32) << 16) | ((hw >> 8) & 0xf) | ((hw >> 13) & 0x7) << 4 |
                                                              ((hw >> 12) & 1) << 7;
    per_cu[cu].push_back({d[7], d[8]});
  }
  std::vector<double> gaps;
  for (auto& [cu, v] : per_cu) {
    std::sort(v.begin(), v.end());
    for (size_t i = 1; i < v.size(); ++i)
      if (v[i].first >= v[i - 1].second) gaps.push_back(static_cast<double>(v[i].first - v[i - 1].second) * 10.0);
  }
  std::fprintf(stderr, "conv1 phases (median clk per workgroup, wave 0, %zu workgroups on %zu CUs):", ph[0].size(),
               per_cu.size());
  for (int i = 0; i < 6; ++i) std::fprintf(stderr, " %s %.0f;", names[i], median(ph[i]));
  std::fprintf(stderr, " lifetime %.0f ns; gap to the next workgroup on the CU %.0f ns (median of %zu)\n",
               median(life), median(gaps), gaps.size());
}

hipError_t conv1_fused_launch(const Conv1WinoPlan& w, const float* x, const float* U, const float* bias, OutView out,
                              bool relu, hipStream_t s, float* p1, int Hp, int Wp, int um = 0) {
  static const hipError_t attr = [] {
    for (const void* k : {reinterpret_cast<const void*>(conv1_fused_kernel<false>),
                          reinterpret_cast<const void*>(conv1_fused_kernel<true>),
                          reinterpret_cast<const void*>(conv1_fused_kernel<true, 0, 1>),
                          reinterpret_cast<const void*>(conv1_fused_kernel<true, 0, 2>)}) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }();
  if (attr != hipSuccess) return attr;
  Conv1FusedArgs a{};
  a.x = x;
  a.U = U;
  a.bias = bias;
  a.out = out;
  a.P = w.P;
  a.ty = w.ty;
  a.tx = w.tx;
  a.Ho = w.H1;
  a.Wo = w.W1;
  a.Hin = w.Hin;
  a.rowf = w.W * 3;
  a.xbytes = static_cast<int>(static_cast<long>(w.N) * w.Hin * w.W * 3 * 4);
  a.ubytes = kPts * kK * kCh * 4;
  a.n_ptiles = (w.P + kTiles - 1) / kTiles;
  a.per_xcd = (a.n_ptiles + 7) / 8;
  a.relu = relu ? 1 : 0;
  a.p1 = p1;
  a.Hp = Hp;
  a.Wp = Wp;
  const unsigned grid = static_cast<unsigned>(a.per_xcd * 8);
#ifdef ANX_CONV1_ABL  // cost-probe builds only (CMake ANX_CONV1_ABL=ON): ANX_CONV1_ABL=<bits> picks the probe
  static const int abl = [] {
    const char* e = std::getenv("ANX_CONV1_ABL");
    return e ? std::atoi(e) : 0;
  }();
  if (p1 != nullptr && abl != 0) {
    auto go = [&](auto K) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(K), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      K<<<grid, kNT, kLds, s>>>(a);
    };
    switch (abl) {
      case 1: go(conv1_fused_kernel<true, 1>); break;
      case 2: go(conv1_fused_kernel<true, 2>); break;
      case 3: go(conv1_fused_kernel<true, 3>); break;
      case 4: go(conv1_fused_kernel<true, 4>); break;
      case 8: go(conv1_fused_kernel<true, 8>); break;
      case 16: go(conv1_fused_kernel<true, 16>); break;
      case 24: go(conv1_fused_kernel<true, 24>); break;
      case 32: go(conv1_fused_kernel<true, 32>); break;
      case 7: go(conv1_fused_kernel<true, 7>); break;
      case 63: go(conv1_fused_kernel<true, 63>); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
#endif
  static const bool phases = std::getenv("ANX_CONV1_PHASES") != nullptr;
  if (phases && p1 != nullptr) {  // diagnostics: the stamped kernel, then a per-phase summary on stderr
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv1_fused_kernel<true, 64>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv1_fused_kernel<true, 64, 1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv1_fused_kernel<true, 64, 2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_set = true;
    }
    const size_t nb = static_cast<size_t>(a.n_ptiles) * 10;
    unsigned long long* dbg = nullptr;
    if (hipMalloc(&dbg, nb * 8) != hipSuccess) return hipErrorOutOfMemory;
    a.dbg = dbg;
    if (um == 1)
      conv1_fused_kernel<true, 64, 1><<<grid, kNT, kLdsW, s>>>(a);
    else if (um == 2)
      conv1_fused_kernel<true, 64, 2><<<grid, kNT, kLds, s>>>(a);
    else
      conv1_fused_kernel<true, 64><<<grid, kNT, kLds, s>>>(a);
    std::vector<unsigned long long> h(nb);
    hipError_t e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipMemcpy(h.data(), dbg, nb * 8, hipMemcpyDeviceToHost);
    (void)hipFree(dbg);
    if (e != hipSuccess) return e;
    conv1_phase_report(h, a.n_ptiles);
    return hipGetLastError();
  }
  if (p1 != nullptr && um == 1)
    conv1_fused_kernel<true, 0, 1><<<grid, kNT, kLdsW, s>>>(a);
  else if (p1 != nullptr && um == 2)
    conv1_fused_kernel<true, 0, 2><<<grid, kNT, kLds, s>>>(a);

  else if (p1 != nullptr)
    conv1_fused_kernel<true><<<grid, kNT, kLds, s>>>(a);
  else
    conv1_fused_kernel<false><<<grid, kNT, kLds, s>>>(a);
  return hipGetLastError();
}
}  // namespace

hipError_t conv1_fused(const Conv1WinoPlan& w, const float* x, const float* U, const float* bias, OutView out, bool relu,
                       hipStream_t s) {
  if (w.P == 0 || w.H1 <= 0 || w.W1 <= 0) return hipSuccess;
  if (!conv1_fused_eligible(w, out)) return hipErrorInvalidValue;
  return conv1_fused_launch(w, x, U, bias, out, relu, s, nullptr, 0, 0);
}

bool conv1_fused_pool_eligible(const Conv1WinoPlan& w, const OutView& window, int Hp, int Wp) {
  // pooled pixels are decoded from 5 + 5 bits; a window's tiles within kPoolBack raster indices
  // element offsets of both destinations are 32-bit in the epilogue's per-pixel table
  return conv1_fused_eligible(w, window) && w.tx + 1 <= kPoolBack && Hp > 0 && Wp > 0 && Hp <= 32 && Wp <= 32 &&
         2 * Hp + 1 <= w.H1 && 2 * Wp + 1 <= w.W1 && w.N < (1 << 20) &&
         static_cast<long>(w.N) * window.Hb * window.Wb * window.Cb < (1L << 31) &&
         static_cast<long>(w.N) * Hp * Wp * kK < (1L << 31);
}

hipError_t conv1_fused_pool(const Conv1WinoPlan& w, const float* x, const float* U, const float* bias, OutView window,
                            float* p1, int Hp, int Wp, bool relu, hipStream_t s, int um) {
  if (w.P == 0 || w.H1 <= 0 || w.W1 <= 0) return hipSuccess;
  if (p1 == nullptr || !conv1_fused_pool_eligible(w, window, Hp, Wp)) return hipErrorInvalidValue;
  return conv1_fused_launch(w, x, U, bias, window, relu, s, p1, Hp, Wp, um);
}

}  // namespace anx::hip
