// anx/engine.hpp — the Blocks 1-2 inference engine: persistent device weights + workspace,
// full-image forward and the row-tile entry point.
//
// Parity: alexnetForwardPassCUDA (v3_cuda_only/src/alexnet_cuda.cu:22-95) and the public tile
// API alexnetTileForwardCUDA (v4_mpi_cuda/src/alexnet_mpi_cuda.cu:157-205, decl
// v4_mpi_cuda/include/alexnet.hpp:22-25). The reference mallocs 10 buffers and re-uploads the
// weights on every call, all on the default stream; here weights are packed and uploaded once,
// workspace is sized once for `max_batch`, and every call is a pure sequence of kernel launches
// on the caller's stream (capturable into a hipGraph).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "anx/ops.hpp"
#include "anx/plan.hpp"
#include "anx/shapes.hpp"

namespace anx {

enum class Impl : int {
  Mfma = 0,    // MFMA implicit-GEMM convs + fused epilogues (default)
  Direct = 1,  // naive one-thread-per-output kernels (device oracle)
};

// Algorithm for 5x5 stride-1 convolutions (Conv2) on the Mfma path: Auto picks Winograd
// F(3x3,5x5) when eligible and the launch is larger than 8 images (use_winograd), the direct
// implicit GEMM below that. Process-wide; read when a stage is launched.
// WinogradUnfused = input transform + separate batched GEMM (M in HBM) + output transform (A/B).
enum class ConvAlgo : int { Auto = 0, Direct = 1, Winograd = 2, WinogradUnfused = 3 };
void set_conv2_algo(ConvAlgo a);
ConvAlgo conv2_algo();
// Algorithm for Conv1 (stride 4, C = 3) on the Mfma path: Winograd = polyphase Winograd
// F(3x3,3x3) (conv1_wino.hip) when eligible, Auto = that above 8 images per launch, Direct = the implicit-GEMM kernel (bit-identical across
// row decompositions; Winograd tile origins move with the row split, ~1e-7 relative).
void set_conv1_algo(ConvAlgo a);
ConvAlgo conv1_algo();
// Images per launch of stage 1 (Conv1 + Pool1) and stage 2 (Conv2 + Pool2 + LRN); 0 = the whole
// batch (up to the 32-bit-index chunk). Smaller chunks reuse one set of transform/conv buffers per
// chunk, so the Winograd V buffers can stay in the 256 MiB Infinity Cache between the transform that
// writes them and the GEMM that reads them. Process-wide; env ANX_CHUNK1 / ANX_CHUNK2.
void set_stage_chunks(int stage1, int stage2);
// Algorithm actually used by a launch of n images x `rows` output rows of a conv whose full image
// has `full_rows` rows: Auto = Winograd above 8 full images' worth of rows, direct below.
bool use_winograd(ConvAlgo a, int n, int rows, int full_rows);
// Pool1 fused into Conv2's Winograd input transform inside forward()/tile_forward() (the split
// stage1/stage2 path keeps the materialised window for halo exchange). Default off (measured
// slower); ANX_FUSE_POOL1=1 or anx_set_fuse_pool1 enables it.
void set_fuse_pool1(bool on);
bool fuse_pool1();
int stage_chunk(int stage);

struct HostWeights {
  std::vector<float> w1, b1, w2, b2;  // KCFF weights, biases
};

// Deterministic initialisers: constant mode reproduces the reference's golden
// outputs (input 1.0, weights 0.01, bias 0); random mode is a seeded LCG (the reference's V1
// uses rand() seeded by wall-clock, v1_serial/src/main.cpp:12 — not reproducible).
void init_const(HostWeights& w, const BlockSpec& b1, const BlockSpec& b2, float wv = 0.01f, float bv = 0.f);
void init_random(HostWeights& w, const BlockSpec& b1, const BlockSpec& b2, unsigned seed);
void init_input_random(std::vector<float>& x, size_t n, unsigned seed);

class BlocksEngine {
 public:
  BlocksEngine(const BlockSpec& b1, const BlockSpec& b2, int H, int W, const HostWeights& w, int max_batch,
               Impl impl = Impl::Mfma);
  ~BlocksEngine();
  BlocksEngine(const BlocksEngine&) = delete;
  BlocksEngine& operator=(const BlocksEngine&) = delete;

  const BlocksDims& dims() const { return d_; }
  int max_batch() const { return max_batch_; }
  Impl impl() const { return impl_; }

  // x: [N, H, W, C0] device; y: [N, Hp2, Wp2, C2] device.
  hipError_t forward(const float* x, int N, float* y, hipStream_t s);

  // Row tile: x holds image rows t.in (N images, [N, t.in.size(), W, C0]); writes output rows
  // t.out to y ([N, t.out.size(), Wp2, C2]). Equivalent to forward() restricted to those rows.
  hipError_t tile_forward(const float* x, int N, const TilePlan& t, float* y, hipStream_t s);

  // Split stages for per-layer halo exchange (V5). stage1 runs conv1+ReLU+pool1 on input rows
  // t.in and writes pool1 rows t.p1 into the conv2 input window (q2_buffer(), window t.q,
  // zero elsewhere). The caller then fills halo rows of the window (q2_row_ptr) and runs stage2.
  hipError_t stage1(const float* x, int N, const TilePlan& t, hipStream_t s);
  hipError_t stage2(int N, const TilePlan& t, float* y, hipStream_t s);
  // Pointer to row `r` (pool1 index space, inside t.q) of image n in the conv2 input window; rows
  // are (Wp1 + 2*P2) * C1 floats with the first P2 pixels of padding, i.e. a full padded row.
  float* q2_row_ptr(const TilePlan& t, int n, int r);
  size_t q2_row_floats() const { return static_cast<size_t>(wq_) * d_.C1; }
  size_t q2_image_stride_floats(const TilePlan& t) const { return static_cast<size_t>(t.q.size()) * q2_row_floats(); }

 private:
  hipError_t ensure_window(const TilePlan& t, int N, hipStream_t s);
  hipError_t conv1_chunk(const float* xc, int n, const TilePlan& t, hipStream_t s);
  hipError_t conv2_chunk(int n, const TilePlan& t, const float* qc, float* yc, hipStream_t s);

  BlockSpec b1_, b2_;
  BlocksDims d_;
  int max_batch_;
  int chunk_;  // images per internal launch chunk (32-bit index limits)
  Impl impl_;
  int wq_;     // padded conv2 input width
  // device buffers
  float *w1_ = nullptr, *b1d_ = nullptr, *w2_ = nullptr, *b2d_ = nullptr;  // KCFF (direct path)
  float *w1p_ = nullptr, *w2p_ = nullptr;                                  // packed (MFMA path)
  int *koff1_ = nullptr, *koff2_ = nullptr;
  float *c1_ = nullptr, *q2_ = nullptr, *c2_ = nullptr;  // workspace
  size_t q2_cap_ = 0;
  // zero-state cache for the conv2 window
  int win_lo_ = 1 << 30, win_hi_ = -(1 << 30), win_n_ = -1;
  int plan_key1_ = -1, plan_key2_ = -1;
  // Winograd conv2: transformed weights packed for the batched GEMM + V / M workspaces
  float *u2p_ = nullptr, *wv_ = nullptr, *wm_ = nullptr;
  int* ukoff_ = nullptr;
  int wino_key_ = -1;
  // Winograd conv1: transformed polyphase weights + V workspace (full-height tiles of chunk_ images)
  float *u1w_ = nullptr, *wv1_ = nullptr;
  size_t wv1_cap_ = 0;
  size_t wv_cap_ = 0, wm_cap_ = 0;
  std::vector<float> w1h_, w2h_;  // KCFF host copies for re-packing on geometry change
};

}  // namespace anx
