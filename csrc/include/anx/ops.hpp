// anx/ops.hpp — layer operators: CPU reference kernels and HIP (gfx950) launchers.
//
// Layouts: activations NHWC (channel fastest, the reference's per-image
// HWC plus a batch axis); conv weights KCFF `((k*C+c)*F+fh)*F+fw` as the reference stores them
// (v1_serial/src/layers_serial.cpp:70). The fast MFMA path repacks KCFF once into a
// GEMM-friendly [K][F*F*C] image (see ConvPlan) — the reference re-uploads weights every call
// (v4_mpi_cuda/src/alexnet_mpi_cuda.cu:176-191); we keep them resident.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "anx/knobs.hpp"
#include "anx/shapes.hpp"

namespace anx {

// ----------------------------------------------------------------------------------------
// CPU reference kernels (V1 / V2 compute, golden oracle). Parity:
// serialConvLayer/ReluLayer/MaxPoolLayer/LRNLayer (v1_serial/src/layers_serial.cpp:37-175).
// ----------------------------------------------------------------------------------------
namespace cpu {
// y[N,Ho,Wo,K] = conv(x[N,H,W,C], w[K,C/g,F,F]) + b ; zero padding P, stride S, groups g.
// `pad_top`/`pad_bottom` override P on the H axis (row tiles: only global edges are padded).
void conv2d(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C, int K, int F,
            int S, int P, int groups, bool relu, int pad_top = -1, int pad_bottom = -1);
void relu(float* x, size_t n);
void maxpool(const float* x, float* y, int N, int H, int W, int C, int F, int S);
void lrn(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta, float k,
         LrnMode mode);
}  // namespace cpu

// ----------------------------------------------------------------------------------------
// HIP launchers. All take device pointers and a stream; none allocate or synchronise
// (safe under hipGraph capture). Return hipSuccess or the launch error.
// ----------------------------------------------------------------------------------------
namespace hip {

// Naive one-thread-per-output kernels: the device-side correctness oracle (the shape of the
// reference's convKernel/poolKernel/lrnKernel, v3_cuda_only/src/layers_cuda.cu:20-152).
hipError_t conv2d_direct(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C,
                         int K, int F, int S, int P, int groups, bool relu, hipStream_t s);
hipError_t relu(float* x, size_t n, hipStream_t s);
hipError_t maxpool_direct(const float* x, float* y, int N, int H, int W, int C, int F, int S, hipStream_t s);
hipError_t lrn_direct(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta,
                      float k, LrnMode mode, hipStream_t s);

// A strided NHWC destination: element (n,h,w,c) of the logical output lands at
// base + ((n*Hb + h + h_off)*Wb + w + w_off)*Cb + c_off + c. Lets producers write straight into
// the zero-bordered input buffer of the next conv (no pad pass) or into a channel slice.
struct OutView {
  float* base;
  int Hb, Wb, Cb;
  int h_off, w_off, c_off;
};

// Implicit-GEMM convolution on f32 MFMA (v_mfma_f32_32x32x2_f32), LDS-staged, fused
// bias + optional ReLU epilogue. The input buffer must already hold the zero padding
// (Hp = H + pads): the kernel performs no bounds checks on reads.
struct ConvPlan {
  int N, Hp, Wp, C;   // padded input dims
  int K, F, S, groups;
  int Ho, Wo;         // output dims
  int Cg, Kg;         // per-group channels / filters
  int kdim;           // F*F*Cg (real)
  int kpad;           // kdim rounded up to BK
  int kpad_n;         // Kg rounded up to BN
  int variant;        // tile configuration id
  int vec4;           // A is gathered in 4-float units (16-B loads)
  int taps4;          // Cg%4 != 0 (conv1, C=3): each filter row's F*C contiguous floats are cut
                      // into 4-float units, the last one shifted back to end at F*C (its
                      // overlap gets zero weight) -> kdim = F*4*ceil(F*C/4), 16-B gathers
};
// force_vec4 / force_scalar: tile variant override for Cg%4==0 / scalar-gather convs (A/B tuning,
// Knobs::force_vec4 / force_scalar; -1 or an invalid id = the heuristic).
ConvPlan make_conv_plan(int N, int Hp, int Wp, int C, int K, int F, int S, int groups, int force_vec4 = -1,
                        int force_scalar = -1);
bool conv_variant_valid(int kind, int id);
// Packed weights: [groups][kpad_n][kpad] with k = (fh*F + fw)*Cg + c (taps4: k = (fh*U + u)*4 + e
// over the 4-float units u of filter row fh); zero padded.
size_t packed_weight_floats(const ConvPlan& p);
// Offset table: [kpad] int32 input offsets (relative to the pixel's window origin), -1 = padding.
size_t koff_ints(const ConvPlan& p);
// Host-side packing (weights come from the host in KCFF order).
void pack_conv_weights_host(const ConvPlan& p, const float* w_kcff, std::vector<float>& packed,
                            std::vector<int>& koff);
hipError_t conv2d_mfma(const ConvPlan& p, const float* x, const float* wpacked, const int* koff,
                       const float* bias, OutView out, bool relu, hipStream_t s);

// Winograd F(m x m, 5x5) for stride-1 5x5 convolutions over a pre-padded input window (winograd.hip):
// m = 3 (7x7 input tiles, 49 points) or m = 4 (8x8, 64 points; Knobs::conv2_tile).
struct WinoPlan {
  int N, Hq, Wq, C, K, groups;
  int Ho, Wo, ty, tx, P;  // output dims, m x m tiles per column/row, total tiles
  int m;                  // output tile side
};
// m = 3: 96 or 48 channels per group and a multiple of 64 filters per group; m = 4: one group, 96
// channels, a multiple of 64 filters (the fused GEMMs' shapes)
bool wino_eligible(int F, int S, int C, int K, int groups, int m = 3);
WinoPlan make_wino_plan(int N, int Hq, int Wq, int C, int K, int groups, int m = 3);
size_t wino_v_floats(const WinoPlan& w);  // V workspace [P][(m+4)^2][C]
size_t wino_u_floats(const WinoPlan& w);  // transformed weights [(m+4)^2][K][C/groups]
// U[(ab*groups + g)*Kg + k][c] = (G g G^T)[a][b] in fp64, rounded once.
void wino_transform_weights_host(const WinoPlan& w, const float* w_kcff, std::vector<float>& u_kcff);
hipError_t wino_input(const WinoPlan& w, const float* x, float* V, hipStream_t s);
// Pool1 (3x3 / 2 max) fused with the input transform: V straight from the conv1 output c1 [N][H1][W1][C]
// (conv1 row c1_lo first). Window row R is pool1 row q_lo + R (zero outside [0, Hp)), window column c is
// pool1 column c - P (zero outside [0, Wp)); every non-zero window row must be computable from c1's rows.
// Bit-identical to maxpool + wino_input. C % 32 == 0, Wq <= 31, and the pooling must be 3x3 / stride 2
// (pool_F, pool_S; anything else returns hipErrorInvalidValue: the kernel's walk is written for 3/2).
hipError_t wino_pool_input(const WinoPlan& w, const float* c1, int H1, int W1, int q_lo, int Hp, int Wp, int P,
                           int c1_lo, float* V, hipStream_t s, int pool_F = 3, int pool_S = 2);
// Input transform of a conv2 window whose pool1 pixels were written by conv1_fused_pool: straddling
// pixels take max(window, p1) (p1: [N][Hp][Wp][C], image 0 = tile-numbering image n_off of the Conv1
// launch with ty1 x tx1 tiles per image). Window row R is pool1 row q_lo + R, column c pool1 column c - P.
// pg: channels per workgroup, 32 (31 KiB of LDS, 512 threads) or 16 (15.5 KiB, 256 threads: fits beside a
// Conv1 workgroup of the per-wave-ring kernel, 142 KiB, on one CU; knob conv2_in_pg).
hipError_t wino_window_merge_input(const WinoPlan& w, const float* window, const float* p1, int n_off, int ty1, int tx1,
                                   int q_lo, int Hp, int Wp, int P, float* V, hipStream_t s, int pg = 32);
// Fused batched GEMM + output transform + bias + optional ReLU into `out` (wino_gemm.hpp); Knobs:
// conv2_occ (workgroups per CU cap).
hipError_t wino_conv2(const WinoPlan& w, const float* V, const float* U, const float* bias, OutView out, bool relu,
                      hipStream_t s, const Knobs& k);

// Conv1 (stride 4, C = 3, 8 < F <= 12, no padding) as Winograd F(3x3,3x3) on the polyphase image
// (conv1_wino.hip): 48 polyphase channels, 3x3 output tiles, 25 transform points.
struct Conv1WinoPlan {
  int N, Hin, W, K, F;
  int H1, W1, ty, tx, P;  // output dims, 3x3 tiles per column/row, total tiles
};
bool conv1_wino_eligible(int C, int K, int F, int S, int P, int groups);
Conv1WinoPlan make_conv1_wino_plan(int N, int Hin, int W, int K, int F);
size_t conv1_wino_v_floats(const Conv1WinoPlan& w);  // V workspace [P][25][48]
size_t conv1_wino_u_floats(int K);                   // transformed weights [25][K][48]
void conv1_wino_weights_host(int K, int F, const float* w_kcff, std::vector<float>& u);
// x: [N, Hin, W, 3] image rows; writes conv1 (+bias, optional ReLU) through `out`. Knobs: conv1_occ,
// conv1_band, conv1_fused (1 / 2: the one-kernel form below instead of transform kernel + GEMM).
hipError_t conv1_wino(const Conv1WinoPlan& w, const float* x, float* V, const float* U, const float* bias, OutView out,
                      bool relu, hipStream_t s, const Knobs& k);
// The one-kernel form (conv1_fused.hip): the input transform generated in LDS inside the GEMM, each
// workgroup 32 tiles x all 96 filters (V never reaches HBM, U through an LDS-DMA ring). Eligible for
// K == 96.
bool conv1_fused_eligible(const Conv1WinoPlan& w, const OutView& out);
hipError_t conv1_fused(const Conv1WinoPlan& w, const float* x, const float* U, const float* bias, OutView out, bool relu,
                       hipStream_t s);
// The same kernel with pool1 (3x3 / 2 max) in its epilogue: the 55x55 conv1 map never leaves LDS. Pooled
// pixel (py, px) of image n is written to `window` (pool1 image at h_off / w_off, e.g. the conv2 input
// window) by the workgroup owning the window's top-left Conv1 tile; when the window's tiles straddle two
// workgroups' 32-tile ranges (pool1_straddles), that value is the lower workgroup's partial max and the
// upper one's is in p1 [N][Hp][Wp][K]: the consumer takes the max of both (wino_window_merge_input).
// Exact (max in any order), so the merged pool1 map equals conv1_fused + maxpool.
constexpr int kConv1FusedTiles = 32;  // Conv1 tiles per conv1_fused workgroup (raster order)
__host__ __device__ inline bool pool1_straddles(int n, int py, int px, int ty1, int tx1) {
  const int b = n * ty1 * tx1;
  const int gm = b + (2 * py / 3) * tx1 + (2 * px) / 3, gM = b + ((2 * py + 2) / 3) * tx1 + (2 * px + 2) / 3;
  return gm / kConv1FusedTiles != gM / kConv1FusedTiles;
}
bool conv1_fused_pool_eligible(const Conv1WinoPlan& w, const OutView& window, int Hp, int Wp);
hipError_t conv1_fused_pool(const Conv1WinoPlan& w, const float* x, const float* U, const float* bias, OutView window,
                            float* p1, int Hp, int Wp, bool relu, hipStream_t s, int um = 0);

// The fused Winograd GEMM + output transform (wino_gemm.hip). V [P][points][C], U [points][K][C/groups]
// (row = filter), bias + optional ReLU, NHWC store through `out` (Cb, c_off multiples of 4). P tiles of
// 3x3 outputs on a ty x tx grid per image, Ho x Wo outputs. occ: workgroups-per-CU cap (0 = none).
// abl / cfg: 0 / -1 = the production kernel; other ablations and configurations exist only in the
// anx_wgemm A/B build.
hipError_t wino_gemm_conv2(const float* V, const float* U, const float* bias, OutView out, int P, int ty, int tx, int Ho,
                           int Wo, int C, int K, int groups, bool relu, hipStream_t s, int occ = 0, int abl = 0,
                           int cfg = -1);
hipError_t wino_gemm_conv1(const float* V, const float* U, const float* bias, OutView out, int P, int ty, int tx, int Ho,
                           int Wo, int K, bool relu, hipStream_t s, int occ = 0, int abl = 0, int cfg = -1);
// The F(4x4,5x5) form (wino_gemm16.hpp): V [P][64][96], U [64][K][96], P tiles of 4x4 outputs, K % 64 == 0.
// abl 0 = the compiler-scheduled kernel, kConv2SchedAbl = the hand-scheduled slice (knob conv2_sched; bitwise
// identical), other values = A/B-tool probes.
constexpr int kConv2SchedAbl = 64 + 256 + 512;
hipError_t wino_gemm_conv2_f45(const float* V, const float* U, const float* bias, OutView out, int P, int ty, int tx,
                               int Ho, int Wo, int K, bool relu, hipStream_t s, int occ = 0, int abl = 0, int cfg = -1);
// The same GEMM with pool2 (3x3 / 2 max) in its epilogue: the 27x27 conv2 map never reaches HBM. Pooled
// pixel (py, px) of image n goes to pooled [n][Hp][Wp][K] from the workgroup owning the window's top-left
// 4x4 tile (tile (py / 2, px / 2)); when the window's tiles straddle two workgroups' 32-tile ranges
// (pool2_straddles), that value is the lower workgroup's partial max and the upper one's is in p2 (same
// layout): the consumer takes the max of both (lrn_pooled_merge). Exact (max in any order).
constexpr int kConv2PoolTiles = 32;  // Conv2 4x4 tiles per F(4x4,5x5) GEMM workgroup (raster order)
__host__ __device__ inline bool pool2_straddles(int n, int py, int px, int ty2, int tx2) {
  const int gm = n * ty2 * tx2 + (py >> 1) * tx2 + (px >> 1);
  const int gM = gm + ((py & 1) ? tx2 : 0) + (px & 1);
  return gm / kConv2PoolTiles != gM / kConv2PoolTiles;
}
hipError_t wino_gemm_conv2_f45_pool(const float* V, const float* U, const float* bias, float* pooled, float* p2, int P,
                                    int ty, int tx, int Ho, int Wo, int Hp, int Wp, int K, bool relu, hipStream_t s,
                                    int occ = 0, bool sched = false);


// Dynamic LDS bytes that cap a kernel at `wgs` workgroups per CU (160 KiB LDS per CU): the larger of
// `natural` and just over 160 KiB / (wgs + 1). wgs <= 0: `natural`.
size_t occupancy_lds(size_t natural, int wgs);

// Vectorised NHWC max-pool writing through an OutView (C % 4 == 0 required for the fast path).
hipError_t maxpool(const float* x, int N, int H, int W, int C, int F, int S, OutView out, hipStream_t s);
// Fused max-pool + cross-channel LRN (block 2 tail).
hipError_t maxpool_lrn(const float* x, float* y, int N, int H, int W, int C, int F, int S, int size,
                       float alpha, float beta, float k, LrnMode mode, hipStream_t s);
// LRN of a pooled map written by wino_gemm_conv2_f45_pool (C == 256, size 5): pixel (n, py, px) is
// max(pooled, p2) where pool2_straddles(n % sub, ...) (sub: images per GEMM launch, ty2 x tx2 tiles per
// image), pooled alone elsewhere. Bit-identical to maxpool_lrn of the unpooled map. max_wgs > 0 caps the
// grid (knob lrn_wgs: each wave then walks several pixel pairs; same output bits).
hipError_t lrn_pooled_merge(const float* pooled, const float* p2, float* y, int N, int Hp, int Wp, int C, int ty2,
                            int tx2, int sub, int size, float alpha, float beta, float k, LrnMode mode, hipStream_t s,
                            int max_wgs = 0);

// Zero the rows of an NHWC buffer outside [row_lo, row_hi) and the W border (halo buffers).
hipError_t fill(float* x, size_t n, float v, hipStream_t s);
// 16-B-vector copy on exactly `workgroups` workgroups (the ingest probe's stand-in for a collective's
// receive channels: tools/probe_ingest.py). bytes % 16 == 0, both pointers 16-B aligned.
hipError_t channel_copy(void* dst, const void* src, size_t bytes, int workgroups, hipStream_t s);

}  // namespace hip
}  // namespace anx
