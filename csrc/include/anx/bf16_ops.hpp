// anx/bf16_ops.hpp — bf16 MFMA kernels of the full-AlexNet extension (conv_bf16.hip) and the
// full-network engine (full_engine.cpp). Activations are bf16 NHWC, accumulation fp32.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "anx/knobs.hpp"
#include "anx/shapes.hpp"

namespace anx {
namespace hip {

struct OutViewB {
  __bf16* base;
  int Hb, Wb, Cb;
  int h_off, w_off, c_off;
};

struct ConvPlanB {
  int N, Hp, Wp, C, K, F, S, groups;
  int Ho, Wo, Cg, Kg, kdim, kpad, kpad_n, variant, vec8;
  int taps8;  // C%8 != 0 (conv1): each filter row's F*C contiguous bf16 cut into 8-element units,
              // the last shifted back to end at F*C (overlap zero-weighted) -> 16-B gathers
};

uint16_t f32_to_bf16_bits(float f);
ConvPlanB make_conv_plan_bf16(int N, int Hp, int Wp, int C, int K, int F, int S, int groups);
size_t packed_weight_elems_bf16(const ConvPlanB& p);
void pack_conv_weights_bf16(const ConvPlanB& p, const float* w_kcff, std::vector<uint16_t>& packed,
                            std::vector<int>& koff);
// Split-K for the fully-connected layers (1x1 "convs" with M = batch): ksplit K slices write fp32
// partial slabs [ksplit][M][K] to ws, splitk_reduce_bf16 sums them + bias (+ReLU) into the output.
struct SplitK {
  int ksplit = 1;
  float* ws = nullptr;
};
int fc_split_k(const ConvPlanB& p);  // chosen slice count (1 = no split)
hipError_t splitk_reduce_bf16(const float* ws, int ksplit, int M, int K, const float* bias, bool relu, OutViewB out,
                              float* out_f32, hipStream_t s);
// out_f32 != nullptr: write fp32 (contiguous [M][K]) instead of the bf16 view (final logits).
// glds (Knobs::bf16_glds): 128x128 vec8 layers (conv2-5, FC) run the LDS-DMA ring with 2 (default) or
// 3 slots, 0 = the register-staged kernel (A/B).
hipError_t conv2d_bf16(const ConvPlanB& p, const void* x, const void* wpacked, const int* koff, const float* bias,
                       OutViewB out, float* out_f32, bool relu, hipStream_t s, SplitK split = {}, int glds = 2);
// Wide-tile kernel (conv_bf16_big.hip): 1 workgroup per CU, 8 waves over a 256-row tile, LDS-DMA
// double buffer, 16x16x32 MFMA, LDS-transposed epilogue with 16-B stores. Same packed weights / koff
// as conv2d_bf16 (vec8, non-taps8 plans; the koff table is recomputed in arithmetic); bf16 output
// only. cfg (BM x BN, waves, LDS stages): 0 = 256x256 8w 2, 1 = 256x128 8w 2, 2 = 256x96 8w 2,
// 3 = 128x128 4w 2, 4 = 128x96 4w 2, 5 = 256x128 8w 3, 6 = 128x128 4w 3, 7 = 128x96 4w 3,
// 8 = 256x64 8w 3 (FC); 0, 3, 4 read both k-steps' fragments ahead of their MFMAs (PIPE), 9-11 are
// those three without it (A/B); 12 / 13 = 256x256 / 256x128 ping-pong (two staggered 4-wave
// groups; A 2 / B 3 stages; conv only).
int conv_bf16_big_cfgs();
constexpr int kConvBf16BigCfgs = 17;  // == conv_bf16_big_cfgs() (static_assert in conv_bf16_big.hip); knob range
bool conv_bf16_big_ok(const ConvPlanB& p, int cfg, const OutViewB& out);
// The config a cost model of wave quantization picks for this launch (-1: none applies).
int pick_bf16_big_cfg(const ConvPlanB& p, const OutViewB& out, int cus = 256);
// split.ws set (groups == 1): fp32 partial slabs [ksplit][M][Kg] into split.ws, K split ksplit ways
// (no bias / ReLU; then splitk_reduce_bf16, which also serves an fp32 result at ksplit 1). `out` is
// then only validated.
hipError_t conv2d_bf16_big(const ConvPlanB& p, int cfg, const void* x, const void* wpacked, const int* koff,
                           const float* bias, OutViewB out, bool relu, hipStream_t s, SplitK split = {});
// Fully-connected layer plan on the wide-tile kernel (cfg -1: not applicable).
struct BigFc {
  int cfg, ksplit;
};
// cfg >= 0 forces that wide-tile config (knob bf16_fc_cfg; -1 = cfg 8, the measured default).
constexpr int kMaxFcSplit = 16;
// min_kt: K tiles per split-K slice at least this many (knob bf16_fc_minkt)
BigFc pick_bf16_big_fc(const ConvPlanB& p, int cus = 256, int cfg = -1, int min_kt = 4);
hipError_t maxpool_bf16(const void* x, int N, int H, int W, int C, int F, int S, OutViewB out, hipStream_t s);
// tile (Knobs::bf16_lrn_tile): 1 = the generic LDS-tile kernel even where the C = 256 wave kernel applies (A/B).
hipError_t maxpool_lrn_bf16(const void* x, int N, int H, int W, int C, int F, int S, int size, float alpha,
                            float beta, float k, LrnMode mode, OutViewB out, hipStream_t s, int tile = 0);
hipError_t f32_to_bf16(const float* x, void* y, size_t n, hipStream_t s);
// Conv1 polyphase input (space-to-depth by the stride 4) fused with the bf16 conversion:
// y[n][i][j][(rh*4+rw)*3+c] = x[n][4i+rh][4j+rw][c] (0 past the image), y = [N, ceil(H/4), ceil(W/4), 48].
hipError_t f32_to_bf16_s2d4(const float* x, void* y, int N, int H, int W, hipStream_t s);
// Conv1 on the polyphase image as a persistent row-band kernel (conv1_bf16_ring.hip): x' [N,57,57,48]
// bf16, weights packed by pack_conv1_ring_weights from the polyphase fp32 filters [96][48][3][3]
// (conv1_ring_weight_bytes() bytes), bias + ReLU (relu must be true), bf16 NHWC out (55x55x96 view).
void pack_conv1_ring_weights(const float* w_k48_33, std::vector<uint16_t>& out);
size_t conv1_ring_weight_bytes();
// f32_input: x is the fp32 NHWC image [N,227,227,3] (space-to-depth + bf16 conversion inside the
// kernel, no polyphase copy); else the polyphase bf16 image of f32_to_bf16_s2d4.
// pool_out: also max-pool 3x3/2 into this 27x27x96 view (pool1). With f32_input and one workgroup
// per image (N >= cus) the pool runs in the kernel's epilogue and `out` is NOT written (the 55x55
// map never reaches HBM); otherwise Conv1 writes `out` (dense 55x55x96) and maxpool_bf16 follows.
hipError_t conv1_bf16_ring(const void* x, int N, const void* wpacked, const float* bias, OutViewB out, bool relu,
                           hipStream_t s, int cus = 256, bool f32_input = false, const OutViewB* pool_out = nullptr);

}  // namespace hip

// Full AlexNet (extension): the reference's Blocks 1-2 followed by the AlexNet tail
// Conv3 3x3/1 p1 (256->384) -> ReLU -> Conv4 (384->384) -> ReLU -> Conv5 (384->256) -> ReLU ->
// MaxPool 3/2 -> FC6 9216->4096 -> ReLU -> FC7 4096->4096 -> ReLU -> FC8 4096->classes.
struct FullWeights {
  // KCFF conv weights / [out][in] FC weights (FC6 input order = NHWC flatten of 6x6x256) + biases
  std::vector<float> w[8], b[8];
};
void full_weight_shapes(int classes, int groups2, size_t wn[8], size_t bn[8]);

class FullEngine {
 public:
  FullEngine(const FullWeights& w, int classes, int max_batch, int groups2 = 1, LrnMode lrn = LrnMode::DivN,
             const Knobs& k = default_knobs());
  ~FullEngine();
  FullEngine(const FullEngine&) = delete;
  FullEngine& operator=(const FullEngine&) = delete;
  // x: [N,227,227,3] fp32 device; logits: [N,classes] fp32 device.
  hipError_t forward(const float* x, int N, float* logits, hipStream_t s, bool mark = false);
  // forward(..., mark = true) records this engine's mark event on `s` once Conv2 + Pool2/LRN of the
  // first chunk are enqueued (about half of the forward): wait_mark makes another stream wait for it,
  // which staggers free-running lanes (AlexNetFull.forward_async) by half a forward.
  hipError_t wait_mark(hipStream_t s) const { return mark_ ? hipStreamWaitEvent(s, mark_, 0) : hipErrorInvalidValue; }
  int classes() const { return classes_; }
  int max_batch() const { return max_batch_; }
  Knobs& knobs() { return k_; }  // read at every launch (bf16_glds, bf16_big)
  // Debug / numerics taps: copy the bf16 activation buffer `i` of the last forward (images of its
  // last chunk; N <= chunk) to dst on stream s. i: 0 conv1 [N,55,55,96], 1 pool1 window
  // [N,31,31,96], 2 conv2 [N,27,27,256], 3 pool2+LRN window [N,15,15,256], 4 conv3 window
  // [N,15,15,384], 5 conv4 window [N,15,15,384], 6 conv5 [N,13,13,256], 7 pool5 [N,9216],
  // 8 fc6 [N,4096], 9 fc7 [N,4096]. Returns the element count per image (0 for a bad i).
  size_t tap(int i, int N, void* dst, hipStream_t s) const;

 private:
  hipEvent_t mark_ = nullptr;
  struct Layer {
    int C, K, F, S, groups;
    void* wp = nullptr;
    int* koff = nullptr;
    float* bias = nullptr;
    int key = -1;
    std::vector<float> host;  // KCFF fp32 (re-pack when the tile variant changes)
  };
  hipError_t conv(Layer& L, int N, int Hp, int Wp, const void* x, hip::OutViewB out, float* out_f32, bool relu,
                  hipStream_t s);
  Layer L_[8];
  Knobs k_;
  int classes_, max_batch_, chunk_;
  int cus_ = 256;  // compute units (the wide-tile kernel's cost model)
  LrnMode lrn_;
  bool poly1_ = false;  // Conv1 as a stride-1 3x3 conv over the 48-channel polyphase image (ANX_FULL_CONV1)
  void* w1ring_ = nullptr;  // Conv1 weights packed for conv1_bf16_ring (poly1_ only)
  void *xb_ = nullptr, *c1_ = nullptr, *q2_ = nullptr, *c2_ = nullptr, *q3_ = nullptr, *q4_ = nullptr,
       *q5_ = nullptr, *c5_ = nullptr, *f6_ = nullptr, *f7_ = nullptr, *f8_ = nullptr;
  float* ws_ = nullptr;  // split-K partial slabs of the FC layers (sized for every batch <= chunk_)
};

}  // namespace anx
