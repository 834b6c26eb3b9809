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

#include "anx/knobs.hpp"
#include "anx/ops.hpp"
#include "anx/plan.hpp"
#include "anx/shapes.hpp"

namespace anx {

enum class Impl : int {
  Mfma = 0,    // MFMA implicit-GEMM convs + fused epilogues (default)
  Direct = 1,  // naive one-thread-per-output kernels (device oracle)
};

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
  // k: kernel selection and tuning of this engine (default_knobs(): built-in defaults + ANX_* env).
  BlocksEngine(const BlockSpec& b1, const BlockSpec& b2, int H, int W, const HostWeights& w, int max_batch,
               Impl impl = Impl::Mfma, const Knobs& k = default_knobs());
  ~BlocksEngine();
  BlocksEngine(const BlocksEngine&) = delete;
  BlocksEngine& operator=(const BlocksEngine&) = delete;

  const BlocksDims& dims() const { return d_; }
  int max_batch() const { return max_batch_; }
  Impl impl() const { return impl_; }
  // Read at every launch: changing a knob between calls switches kernels. Use set_knob (it prepares
  // the weights / workspace the new setting needs outside any forward); a field written through
  // knobs() directly re-packs direct-path weights lazily and runs a conv without its Winograd workspace
  // on the direct path. set_knob is a between-forwards operation: a change of conv2_tile or a conv algo
  // frees and re-allocates transformed weights / workspaces, so a HIP graph captured before it (bench
  // --graph) names freed buffers and must be re-captured. Throws (knobs restored) when a re-allocation fails.
  const Knobs& knobs() const { return k_; }
  int set_knob(const char* name, int value);  // 0, or -1 for a bad name / value (unchanged)

  // x: [N, H, W, C0] device; y: [N, Hp2, Wp2, C2] device.
  hipError_t forward(const float* x, int N, float* y, hipStream_t s);

  // Row tile: x holds image rows t.in (N images, [N, t.in.size(), W, C0]); writes output rows
  // t.out to y ([N, t.out.size(), Wp2, C2]). Equivalent to forward() restricted to those rows.
  hipError_t tile_forward(const float* x, int N, const TilePlan& t, float* y, hipStream_t s);

  // Split stages for per-layer halo exchange (V5). stage1 runs conv1+ReLU+pool1 on input rows
  // t.in and writes pool1 rows t.p1 into the conv2 input window (q2_buffer(), window t.q,
  // zero elsewhere). The caller then fills halo rows of the window (q2_row_ptr) and runs stage2.
  // [n_lo, n_hi) restricts either stage to those images of the N-image buffers (x / y / window
  // still address image 0): the V5 runtime pipelines the halo exchange over such image chunks.
  hipError_t stage1(const float* x, int N, const TilePlan& t, hipStream_t s, int n_lo = 0, int n_hi = -1);
  hipError_t stage2(int N, const TilePlan& t, float* y, hipStream_t s, int n_lo = 0, int n_hi = -1);
  // Pointer to row `r` (pool1 index space, inside t.q) of image n in the conv2 input window; rows
  // are (Wp1 + 2*P2) * C1 floats with the first P2 pixels of padding, i.e. a full padded row.
  float* q2_row_ptr(const TilePlan& t, int n, int r);
  size_t q2_row_floats() const { return static_cast<size_t>(wq_) * d_.C1; }
  size_t q2_image_stride_floats(const TilePlan& t) const { return static_cast<size_t>(t.q.size()) * q2_row_floats(); }

 private:
  void prepare();
  hipError_t pack1(const hip::ConvPlan& p);  // direct-path packed weights for plan p (no-op when current)
  hipError_t pack2(const hip::ConvPlan& p);
  hipError_t ensure_window(const TilePlan& t, int N, hipStream_t s);
  // conv1 (+ReLU) of n images into c1_ starting at image c1_img0
  hipError_t conv1_chunk(const float* xc, int n, const TilePlan& t, hipStream_t s, int c1_img0 = 0);
  hipError_t conv2_chunk(int n, const TilePlan& t, const float* qc, float* yc, hipStream_t s);
  hipError_t pool2_chunk(int n, const TilePlan& t, float* yc, hipStream_t s);  // c2_ -> y (+LRN)
  // Whether tile_forward of N images runs pool1 inside the Winograd input transform (Knobs::fuse_pool1)
  bool fused_pool1(int N, const TilePlan& t) const;
  // ... and whether pool1 runs inside the one-kernel Conv1 instead (Knobs::conv1_pool; whole images only)
  bool conv1_pools(int N, const TilePlan& t) const;
  bool conv2_pools(const TilePlan& t) const;  // pool2 in the F(4x4,5x5) GEMM's epilogue (Knobs::conv2_pool)
  hipError_t tile_forward_conv1_pool(const float* x, int N, const TilePlan& t, float* y, hipStream_t s);

  BlockSpec b1_, b2_;
  BlocksDims d_;
  int max_batch_;
  int chunk_;  // images per internal launch chunk (32-bit index limits)
  Impl impl_;
  Knobs k_;
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
  // Winograd conv2: transformed weights [49][K][C/groups] + V workspace
  float *u2w_ = nullptr, *wv_ = nullptr;
  size_t wv_cap_ = 0;
  int u2_m_ = 3;       // Winograd output tile of u2w_ / wv_ (Knobs::conv2_tile when eligible)
  int tile2() const;   // the tile the knobs ask for and Conv2's shape allows
  // Winograd conv1: transformed polyphase weights + V workspace (full-height tiles of chunk_ images)
  float *u1w_ = nullptr, *wv1_ = nullptr;
  size_t wv1_cap_ = 0;
  std::vector<float> w1h_, w2h_;  // KCFF host copies for re-packing on geometry change
};

}  // namespace anx
