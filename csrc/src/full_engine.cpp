// Full AlexNet engine (bf16 extension, see anx/bf16_ops.hpp). Weights are packed to bf16 once and
// stay resident; every activation between layers lives in a persistent bf16 workspace, with the
// padded layers' inputs kept as zero-bordered windows that the producing kernel writes into.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "anx/bf16_ops.hpp"
#include "anx/upload.hpp"

#define ANX_TRY(expr)                \
  do {                               \
    hipError_t _e = (expr);          \
    if (_e != hipSuccess) return _e; \
  } while (0)

namespace anx {

namespace {
void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void* dalloc(size_t bytes) {
  void* p = nullptr;
  check(hipMalloc(&p, std::max<size_t>(bytes, 16)), "hipMalloc");
  return p;
}
// C, K, F, S per layer (groups filled in per instance for conv2)
constexpr int kGeom[8][4] = {{3, 96, 11, 4},      {96, 256, 5, 1},    {256, 384, 3, 1},   {384, 384, 3, 1},
                             {384, 256, 3, 1},    {9216, 4096, 1, 1}, {4096, 4096, 1, 1}, {4096, 0, 1, 1}};
}  // namespace

void full_weight_shapes(int classes, int groups2, size_t wn[8], size_t bn[8]) {
  for (int i = 0; i < 8; ++i) {
    const int C = kGeom[i][0], K = i == 7 ? classes : kGeom[i][1], F = kGeom[i][2];
    const int g = i == 1 ? groups2 : 1;
    wn[i] = static_cast<size_t>(K) * (C / g) * F * F;
    bn[i] = static_cast<size_t>(K);
  }
}

FullEngine::FullEngine(const FullWeights& w, int classes, int max_batch, int groups2, LrnMode lrn, const Knobs& kn)
    : k_(kn), classes_(classes), max_batch_(max_batch), lrn_(lrn) {
  size_t wn[8], bn[8];
  full_weight_shapes(classes, groups2, wn, bn);
  for (int i = 0; i < 8; ++i) {
    if (w.w[i].size() != wn[i] || w.b[i].size() != bn[i])
      throw std::invalid_argument("full AlexNet: weight " + std::to_string(i) + " has the wrong size");
    Layer& L = L_[i];
    L.C = kGeom[i][0];
    L.K = i == 7 ? classes : kGeom[i][1];
    L.F = kGeom[i][2];
    L.S = kGeom[i][3];
    L.groups = i == 1 ? groups2 : 1;
    L.host = w.w[i];
    L.bias = static_cast<float*>(dalloc(bn[i] * 4));
    check(upload_h2d(L.bias, w.b[i].data(), bn[i] * 4), "H2D bias");
  }
  // Conv1 polyphase (the fp32 Winograd Conv1's rewrite, conv1_wino.hip): space-to-depth by the stride
  // turns 11x11/4 over 3 channels into 3x3/1 over 48, so the implicit GEMM's A gathers are aligned
  // 16-B channel runs instead of taps8's 2-byte-aligned 11-tap rows. Exact: W'[k][(rh*4+rw)*3+c][qh][qw]
  // = w[k][c][4qh+rh][4qw+rw], 0 past the 11x11 window. ANX_FULL_CONV1=taps8 keeps the direct form.
  {
    const char* e = std::getenv("ANX_FULL_CONV1");
    poly1_ = !(e && std::string(e) == "taps8");
  }
  if (poly1_) {
    Layer& L = L_[0];
    std::vector<float> wp(static_cast<size_t>(L.K) * 48 * 9, 0.f);
    for (int k = 0; k < L.K; ++k)
      for (int rh = 0; rh < 4; ++rh)
        for (int rw = 0; rw < 4; ++rw)
          for (int c = 0; c < 3; ++c)
            for (int qh = 0; qh < 3; ++qh)
              for (int qw = 0; qw < 3; ++qw) {
                const int fh = 4 * qh + rh, fw = 4 * qw + rw;
                if (fh < 11 && fw < 11)
                  wp[((static_cast<size_t>(k) * 48 + (rh * 4 + rw) * 3 + c) * 3 + qh) * 3 + qw] =
                      L.host[((static_cast<size_t>(k) * 3 + c) * 11 + fh) * 11 + fw];
              }
    L.host = std::move(wp);
    L.C = 48;
    L.F = 3;
    L.S = 1;
    std::vector<uint16_t> rp;
    hip::pack_conv1_ring_weights(L.host.data(), rp);
    w1ring_ = dalloc(rp.size() * 2);
    check(upload_h2d(w1ring_, rp.data(), rp.size() * 2), "H2D conv1 ring weights");
  }
  {
    int dev = 0;
    check(hipGetDevice(&dev), "hipGetDevice");
    check(hipDeviceGetAttribute(&cus_, hipDeviceAttributeMultiprocessorCount, dev), "CU count");
  }
  chunk_ = std::max(1, std::min(max_batch, static_cast<int>(((1UL << 31) - 1) / (55UL * 55 * 96))));
  const size_t n = static_cast<size_t>(chunk_);
  xb_ = dalloc(n * std::max(227 * 227 * 3, 57 * 57 * 48) * 2);
  c1_ = dalloc(n * 55 * 55 * 96 * 2);
  q2_ = dalloc(n * 31 * 31 * 96 * 2);
  c2_ = dalloc(n * 27 * 27 * 256 * 2);
  q3_ = dalloc(n * 15 * 15 * 256 * 2);
  q4_ = dalloc(n * 15 * 15 * 384 * 2);
  q5_ = dalloc(n * 15 * 15 * 384 * 2);
  c5_ = dalloc(n * 13 * 13 * 256 * 2);
  f6_ = dalloc(n * 9216 * 2);
  f7_ = dalloc(n * 4096 * 2);
  f8_ = dalloc(n * 4096 * 2);
  // zero borders of the padded windows once; kernels only ever write the interiors
  check(hipMemset(q2_, 0, n * 31 * 31 * 96 * 2), "memset");
  check(hipMemset(q3_, 0, n * 15 * 15 * 256 * 2), "memset");
  check(hipMemset(q4_, 0, n * 15 * 15 * 384 * 2), "memset");
  check(hipMemset(q5_, 0, n * 15 * 15 * 384 * 2), "memset");
  size_t ws = 0;  // largest split-K slab set over the FC layers and every batch the engine can see
  for (int i = 5; i < 8; ++i)
    for (int b = 1; b <= chunk_; ++b) {
      const hip::ConvPlanB p = hip::make_conv_plan_bf16(b, 1, 1, L_[i].C, L_[i].K, 1, 1, 1);
      const int ks = hip::fc_split_k(p);
      if (ks > 1) ws = std::max(ws, static_cast<size_t>(ks) * b * L_[i].K);
      for (int c = -1; c < hip::conv_bf16_big_cfgs(); ++c) {  // every config bf16_fc_cfg may force
        const hip::BigFc f = hip::pick_bf16_big_fc(p, cus_, c, 1);  // wide-tile FC slabs (ksplit 1 for fp32 logits)
        if (f.cfg >= 0) ws = std::max(ws, static_cast<size_t>(f.ksplit) * b * L_[i].K);
      }
    }
  if (ws) ws_ = static_cast<float*>(dalloc(ws * 4));
}

FullEngine::~FullEngine() {
  if (mark_) (void)hipEventDestroy(mark_);
  for (Layer& L : L_)
    for (void* p : {L.wp, static_cast<void*>(L.koff), static_cast<void*>(L.bias)})
      if (p) (void)hipFree(p);
  for (void* p : {xb_, c1_, q2_, c2_, q3_, q4_, q5_, c5_, f6_, f7_, f8_, static_cast<void*>(ws_), w1ring_})
    if (p) (void)hipFree(p);
}

hipError_t FullEngine::conv(Layer& L, int N, int Hp, int Wp, const void* x, hip::OutViewB out, float* out_f32,
                            bool relu, hipStream_t s) {
  auto B = [](void* q) { return static_cast<__bf16*>(q); };
  const hip::ConvPlanB p = hip::make_conv_plan_bf16(N, Hp, Wp, L.C, L.K, L.F, L.S, L.groups);
  if (p.variant != L.key) {  // pack for this tile variant (first use / batch-size class change)
    std::vector<uint16_t> pk;
    std::vector<int> ko;
    hip::pack_conv_weights_bf16(p, L.host.data(), pk, ko);
    if (L.wp) ANX_TRY(hipFree(L.wp));
    if (L.koff) ANX_TRY(hipFree(L.koff));
    ANX_TRY(hipMalloc(&L.wp, pk.size() * 2));
    ANX_TRY(hipMalloc(&L.koff, ko.size() * 4));
    ANX_TRY(upload_h2d(L.wp, pk.data(), pk.size() * 2));
    ANX_TRY(upload_h2d(L.koff, ko.data(), ko.size() * 4));
    L.key = p.variant;
  }
  const bool fc = p.Hp == 1 && p.Wp == 1 && p.F == 1;
  if (fc && k_.bf16_big != -2) {  // wide-tile FC: one 256-row tile of the batch, K split over the CUs
    hip::BigFc f = hip::pick_bf16_big_fc(p, cus_, k_.bf16_fc_cfg, k_.bf16_fc_minkt);
    if (f.cfg >= 0 && k_.bf16_big >= 0 && hip::conv_bf16_big_ok(p, k_.bf16_big, hip::OutViewB{B(ws_), 1, 1, p.Kg, 0, 0, 0}))
      f.cfg = k_.bf16_big;
    if (f.cfg >= 0 && (f.ksplit > 1 || out_f32)) {
      ANX_TRY(hip::conv2d_bf16_big(p, f.cfg, x, L.wp, L.koff, L.bias, hip::OutViewB{B(ws_), 1, 1, p.Kg, 0, 0, 0}, relu,
                                   s, hip::SplitK{f.ksplit, ws_}));
      return hip::splitk_reduce_bf16(ws_, f.ksplit, N, L.K, L.bias, relu, out, out_f32, s);
    }
    if (f.cfg >= 0) return hip::conv2d_bf16_big(p, f.cfg, x, L.wp, L.koff, L.bias, out, relu, s);
  }
  const int ks = hip::fc_split_k(p);
  if (ks > 1) {  // FC layer at a small batch: K split over ~one workgroup per CU, then a reduce
    ANX_TRY(hip::conv2d_bf16(p, x, L.wp, L.koff, L.bias, out, out_f32, relu, s, hip::SplitK{ks, ws_}, k_.bf16_glds));
    return hip::splitk_reduce_bf16(ws_, ks, N, L.K, L.bias, relu, out, out_f32, s);
  }
  if (!fc && !out_f32 && k_.bf16_big != -2) {  // wide-tile kernel: forced config if it applies, else the cost model
    const int cfg = k_.bf16_big >= 0 && hip::conv_bf16_big_ok(p, k_.bf16_big, out) ? k_.bf16_big
                                                                                    : hip::pick_bf16_big_cfg(p, out, cus_);
    if (cfg >= 0) return hip::conv2d_bf16_big(p, cfg, x, L.wp, L.koff, L.bias, out, relu, s);
  }
  return hip::conv2d_bf16(p, x, L.wp, L.koff, L.bias, out, out_f32, relu, s, {}, k_.bf16_glds);
}

hipError_t FullEngine::forward(const float* x, int N, float* logits, hipStream_t s, bool mark) {
  if (mark && !mark_) ANX_TRY(hipEventCreateWithFlags(&mark_, hipEventDisableTiming));
  using hip::OutViewB;
  auto B = [](void* p) { return static_cast<__bf16*>(p); };
  for (int n0 = 0; n0 < N; n0 += chunk_) {
    const int n = std::min(chunk_, N - n0);
    const float* xn = x + static_cast<size_t>(n0) * 227 * 227 * 3;
    bool pooled = false;  // pool1 done with Conv1
    if (poly1_) {
      if (k_.bf16_conv1 == 2) {  // the fp32 image straight into the row-band kernel (no polyphase copy)
        const OutViewB q2v{B(q2_), 31, 31, 96, 2, 2, 0};
        ANX_TRY(hip::conv1_bf16_ring(xn, n, w1ring_, L_[0].bias, OutViewB{B(c1_), 55, 55, 96, 0, 0, 0}, true, s, cus_,
                                     true, k_.bf16_pool1 ? &q2v : nullptr));
        pooled = k_.bf16_pool1 != 0;
      } else {
        ANX_TRY(hip::f32_to_bf16_s2d4(xn, xb_, n, 227, 227, s));
        if (k_.bf16_conv1 == 1)
          ANX_TRY(hip::conv1_bf16_ring(xb_, n, w1ring_, L_[0].bias, OutViewB{B(c1_), 55, 55, 96, 0, 0, 0}, true, s, cus_));
        else
          ANX_TRY(conv(L_[0], n, 57, 57, xb_, OutViewB{B(c1_), 55, 55, 96, 0, 0, 0}, nullptr, true, s));
      }
    } else {
      ANX_TRY(hip::f32_to_bf16(xn, xb_, static_cast<size_t>(n) * 227 * 227 * 3, s));
      ANX_TRY(conv(L_[0], n, 227, 227, xb_, OutViewB{B(c1_), 55, 55, 96, 0, 0, 0}, nullptr, true, s));
    }
    if (!pooled) ANX_TRY(hip::maxpool_bf16(c1_, n, 55, 55, 96, 3, 2, OutViewB{B(q2_), 31, 31, 96, 2, 2, 0}, s));
    ANX_TRY(conv(L_[1], n, 31, 31, q2_, OutViewB{B(c2_), 27, 27, 256, 0, 0, 0}, nullptr, true, s));
    ANX_TRY(hip::maxpool_lrn_bf16(c2_, n, 27, 27, 256, 3, 2, 5, 1e-4f, 0.75f, 2.0f, lrn_,
                                  OutViewB{B(q3_), 15, 15, 256, 1, 1, 0}, s, k_.bf16_lrn_tile));
    if (mark && n0 == 0) ANX_TRY(hipEventRecord(mark_, s));
    ANX_TRY(conv(L_[2], n, 15, 15, q3_, OutViewB{B(q4_), 15, 15, 384, 1, 1, 0}, nullptr, true, s));
    ANX_TRY(conv(L_[3], n, 15, 15, q4_, OutViewB{B(q5_), 15, 15, 384, 1, 1, 0}, nullptr, true, s));
    ANX_TRY(conv(L_[4], n, 15, 15, q5_, OutViewB{B(c5_), 13, 13, 256, 0, 0, 0}, nullptr, true, s));
    ANX_TRY(hip::maxpool_bf16(c5_, n, 13, 13, 256, 3, 2, OutViewB{B(f6_), 6, 6, 256, 0, 0, 0}, s));
    ANX_TRY(conv(L_[5], n, 1, 1, f6_, OutViewB{B(f7_), 1, 1, 4096, 0, 0, 0}, nullptr, true, s));
    ANX_TRY(conv(L_[6], n, 1, 1, f7_, OutViewB{B(f8_), 1, 1, 4096, 0, 0, 0}, nullptr, true, s));
    ANX_TRY(conv(L_[7], n, 1, 1, f8_, OutViewB{nullptr, 1, 1, classes_, 0, 0, 0},
                 logits + static_cast<size_t>(n0) * classes_, false, s));
  }
  return hipSuccess;
}

size_t FullEngine::tap(int i, int N, void* dst, hipStream_t s) const {
  static const size_t kElems[11] = {55 * 55 * 96,   31 * 31 * 96, 27 * 27 * 256, 15 * 15 * 256,
                                    15 * 15 * 384,  15 * 15 * 384, 13 * 13 * 256, 9216,
                                    4096,           4096,          57 * 57 * 48};
  void* const bufs[11] = {c1_, q2_, c2_, q3_, q4_, q5_, c5_, f6_, f7_, f8_, xb_};
  if (i < 0 || i >= 11 || (i == 10 && !poly1_) || N < 1 || N > chunk_) return 0;
  if (hipMemcpyAsync(dst, bufs[i], kElems[i] * N * 2, hipMemcpyDeviceToDevice, s) != hipSuccess) return 0;
  return kElems[i];
}

}  // namespace anx
