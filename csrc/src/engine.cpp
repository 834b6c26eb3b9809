// Blocks 1-2 engine (see anx/engine.hpp).
#include "anx/engine.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "anx/rng.hpp"
#include "anx/trace.hpp"
#include "anx/upload.hpp"

#define ANX_TRY(expr)                          \
  do {                                         \
    hipError_t _e = (expr);                    \
    if (_e != hipSuccess) return _e;           \
  } while (0)

namespace anx {

namespace {
void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
template <class T>
T* dev_alloc(size_t n) {
  void* p = nullptr;
  if (n == 0) n = 1;
  check(hipMalloc(&p, n * sizeof(T)), "hipMalloc");
  return static_cast<T*>(p);
}
template <class T>
T* dev_upload(const std::vector<T>& h) {
  T* d = dev_alloc<T>(h.size());
  check(upload_h2d(d, h.data(), h.size() * sizeof(T)), "upload H2D");  // pinned staging (anx/upload.hpp)
  return d;
}
}  // namespace

void init_const(HostWeights& w, const BlockSpec& b1, const BlockSpec& b2, float wv, float bv) {
  const ConvSpec &c1 = b1.conv, &c2 = b2.conv;
  w.w1.assign(static_cast<size_t>(c1.K) * (c1.C / c1.groups) * c1.F * c1.F, wv);
  w.b1.assign(c1.K, bv);
  w.w2.assign(static_cast<size_t>(c2.K) * (c2.C / c2.groups) * c2.F * c2.F, wv);
  w.b2.assign(c2.K, bv);
}

void init_random(HostWeights& w, const BlockSpec& b1, const BlockSpec& b2, unsigned seed) {
  init_const(w, b1, b2);
  // weights (u - 0.5) * 0.02, biases 0.1 (v1_serial/src/alexnet_serial.cpp:39-57).
  for (size_t i = 0; i < w.w1.size(); ++i) w.w1[i] = (rng::uniform(seed, rng::kW1, i) - 0.5f) * 0.02f;
  for (size_t i = 0; i < w.b1.size(); ++i) w.b1[i] = 0.1f;
  for (size_t i = 0; i < w.w2.size(); ++i) w.w2[i] = (rng::uniform(seed, rng::kW2, i) - 0.5f) * 0.02f;
  for (size_t i = 0; i < w.b2.size(); ++i) w.b2[i] = 0.1f;
}

void init_input_random(std::vector<float>& x, size_t n, unsigned seed) {
  x.resize(n);
  for (size_t i = 0; i < n; ++i) x[i] = rng::uniform(seed, rng::kInput, i) * 0.1f;
}

BlocksEngine::BlocksEngine(const BlockSpec& b1, const BlockSpec& b2, int H, int W, const HostWeights& w,
                           int max_batch, Impl impl, const Knobs& k)
    : b1_(b1), b2_(b2), d_(blocks_dims(H, W, b1, b2)), max_batch_(max_batch), impl_(impl), k_(k) {
  if (b1.conv.P != 0) throw std::invalid_argument("conv1 padding must be 0 (row tiles read raw image rows)");
  if (d_.Hp2 <= 0 || d_.Wp2 <= 0) throw std::invalid_argument("input too small for AlexNet blocks 1-2");
  wq_ = d_.Wp1 + 2 * b2.conv.P;
  const size_t per_img = std::max<size_t>(
      {static_cast<size_t>(H) * W * d_.C0, static_cast<size_t>(d_.H1) * d_.W1 * d_.C1,
       static_cast<size_t>(d_.Hp1 + 2 * b2.conv.P) * wq_ * d_.C1, static_cast<size_t>(d_.H2) * d_.W2 * d_.C2,
       // Winograd conv2 V buffer: 49 transform points x C per 3x3 output tile
       static_cast<size_t>((d_.H2 + 2) / 3) * ((d_.W2 + 2) / 3) * 49 * d_.C1,
       // Winograd conv1 V buffer: 25 points x 48 polyphase channels per 3x3 output tile
       static_cast<size_t>((d_.H1 + 2) / 3) * ((d_.W1 + 2) / 3) * 25 * 48});
  // images per launch: every buffer a kernel addresses stays below 2^31 bytes (the Winograd GEMMs
  // reach their operands through 32-bit buffer offsets)
  chunk_ = static_cast<int>(std::min<size_t>(max_batch, ((1UL << 31) - 1) / (per_img * sizeof(float))));
  if (chunk_ < 1) throw std::invalid_argument("image too large for 32-bit kernel indexing");
  // ANX_ENGINE_PHASES=1: where a cold engine's construction goes (stderr; diagnostics only)
  static const bool phases = [] {
    const char* e = std::getenv("ANX_ENGINE_PHASES");
    return e && *e == '1';
  }();
  auto ms = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = phases ? ms() : 0;
  w1h_ = w.w1;
  w2h_ = w.w2;
  w1_ = dev_upload(w.w1);
  b1d_ = dev_upload(w.b1);
  w2_ = dev_upload(w.w2);
  b2d_ = dev_upload(w.b2);
  const double t1 = phases ? ms() : 0;
  c1_ = dev_alloc<float>(static_cast<size_t>(chunk_) * d_.H1 * d_.W1 * d_.C1);
  q2_cap_ = static_cast<size_t>(max_batch) * (d_.Hp1 + 2 * b2.conv.P) * wq_ * d_.C1;
  q2_ = dev_alloc<float>(q2_cap_);
  c2_ = dev_alloc<float>(static_cast<size_t>(chunk_) * d_.H2 * d_.W2 * d_.C2);
  const double t2 = phases ? ms() : 0;
  prepare();
  if (phases)
    std::fprintf(stderr, "ANX_ENGINE_PHASES uploads %.3f allocs %.3f prepare %.3f ms (max_batch %d)\n", t1 - t0, t2 - t1,
                 ms() - t2, max_batch);
}

// What the current knobs can launch, prepared outside any forward (no allocation, upload or host
// packing inside one): the Winograd transformed weights and workspaces only if some launch of up to
// max_batch images can run Winograd (a batch-1 engine under Auto never does: the V3 cold path skips
// both transforms, 2.6 MB of U and the V buffers), and the direct path's packed weights for its
// largest full-image launch (the one a batch-1 engine runs first), so the first forward packs nothing.
void BlocksEngine::prepare() {
  if (impl_ != Impl::Mfma) return;
  const ConvSpec &k1 = b1_.conv, &k2 = b2_.conv;
  if (u1w_ == nullptr && hip::conv1_wino_eligible(k1.C, k1.K, k1.F, k1.S, k1.P, k1.groups) &&
      use_winograd(k_.conv1_algo, max_batch_, d_.H1, d_.H1)) {
    const hip::Conv1WinoPlan wp = hip::make_conv1_wino_plan(chunk_, d_.H, d_.W, k1.K, k1.F);
    std::vector<float> u;
    hip::conv1_wino_weights_host(k1.K, k1.F, w1h_.data(), u);
    // both buffers or neither (a failed allocation leaves the path off and retryable)
    float* v = dev_alloc<float>(hip::conv1_wino_v_floats(wp));
    try {
      u1w_ = dev_upload(u);
    } catch (...) {
      (void)hipFree(v);
      throw;
    }
    wv1_cap_ = hip::conv1_wino_v_floats(wp);
    wv1_ = v;
  }
  if (u2w_ != nullptr && u2_m_ != tile2()) {  // the tile knob changed: other transformed weights / workspace
    for (float** q : {&u2w_, &wv_})
      if (*q) (void)hipFree(*q), *q = nullptr;
    wv_cap_ = 0;
  }
  if (u2w_ == nullptr && hip::wino_eligible(k2.F, k2.S, d_.C1, d_.C2, k2.groups) &&
      use_winograd(k_.conv2_algo, max_batch_, d_.H2, d_.H2)) {
    // Winograd workspace for a full-height window of chunk_ images (row tiles need less)
    const hip::WinoPlan wp = hip::make_wino_plan(chunk_, d_.Hp1 + 2 * k2.P, wq_, d_.C1, d_.C2, k2.groups, tile2());
    u2_m_ = wp.m;
    if (hip::wino_v_floats(wp) < (1UL << 31)) {
      std::vector<float> u;
      hip::wino_transform_weights_host(wp, w2h_.data(), u);
      float* v = dev_alloc<float>(hip::wino_v_floats(wp));
      try {
        u2w_ = dev_upload(u);
      } catch (...) {
        (void)hipFree(v);
        throw;
      }
      wv_cap_ = hip::wino_v_floats(wp);
      wv_ = v;
    }
  }
  // direct path: the full-image launch of min(max_batch, the Auto crossover) images
  static const bool phases = [] {
    const char* e = std::getenv("ANX_ENGINE_PHASES");
    return e && *e == '1';
  }();
  auto ms = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double tp = phases ? ms() : 0;
  const int n = std::max(1, std::min(max_batch_, chunk_));
  const int nd = k_.conv1_algo == ConvAlgo::Direct ? n : std::min(n, 8);
  if (!use_winograd(k_.conv1_algo, nd, d_.H1, d_.H1) || wv1_ == nullptr)
    (void)pack1(hip::make_conv_plan(nd, d_.H, d_.W, d_.C0, k1.K, k1.F, k1.S, k1.groups, k_.force_vec4, k_.force_scalar));
  const int nd2 = k_.conv2_algo == ConvAlgo::Direct ? n : std::min(n, 8);
  if (!use_winograd(k_.conv2_algo, nd2, d_.H2, d_.H2) || wv_ == nullptr)
    (void)pack2(hip::make_conv_plan(nd2, d_.Hp1 + 2 * k2.P, wq_, d_.C1, k2.K, k2.F, k2.S, k2.groups, k_.force_vec4,
                                    k_.force_scalar));
  if (phases) std::fprintf(stderr, "ANX_ENGINE_PHASES direct-path packing %.3f ms\n", ms() - tp);
}

int BlocksEngine::tile2() const {
  const ConvSpec& k2 = b2_.conv;
  return k_.conv2_tile == 4 && hip::wino_eligible(k2.F, k2.S, d_.C1, d_.C2, k2.groups, 4) ? 4 : 3;
}

int BlocksEngine::set_knob(const char* name, int value) {
  const Knobs before = k_;
  if (anx::set_knob(k_, name, value) != 0) return -1;
  try {
    prepare();  // a knob may enable a path whose weights / workspace this engine has not built yet
  } catch (...) {
    // e.g. hipMalloc OOM building a Winograd workspace: keep the previous selection. prepare() builds
    // lazily and a path whose buffers are null is not taken, so the engine stays usable; the caller
    // (anx_engine_set_knob) turns the exception into an error code
    k_ = before;
    throw;
  }
  return 0;
}

hipError_t BlocksEngine::pack1(const hip::ConvPlan& p) {
  const int key = p.variant | (p.taps4 << 8);
  if (key == plan_key1_) return hipSuccess;
  std::vector<float> packed;
  std::vector<int> koff;
  hip::pack_conv_weights_host(p, w1h_.data(), packed, koff);
  if (w1p_) ANX_TRY(hipFree(w1p_));
  if (koff1_) ANX_TRY(hipFree(koff1_));
  w1p_ = dev_upload(packed);
  koff1_ = dev_upload(koff);
  plan_key1_ = key;
  return hipSuccess;
}

hipError_t BlocksEngine::pack2(const hip::ConvPlan& p) {
  const int key = p.variant | (p.taps4 << 8);
  if (key == plan_key2_) return hipSuccess;
  std::vector<float> packed;
  std::vector<int> koff;
  hip::pack_conv_weights_host(p, w2h_.data(), packed, koff);
  if (w2p_) ANX_TRY(hipFree(w2p_));
  if (koff2_) ANX_TRY(hipFree(koff2_));
  w2p_ = dev_upload(packed);
  koff2_ = dev_upload(koff);
  plan_key2_ = key;
  return hipSuccess;
}

BlocksEngine::~BlocksEngine() {
  for (void* p : {static_cast<void*>(w1_), static_cast<void*>(b1d_), static_cast<void*>(w2_),
                  static_cast<void*>(b2d_), static_cast<void*>(w1p_), static_cast<void*>(w2p_),
                  static_cast<void*>(koff1_), static_cast<void*>(koff2_), static_cast<void*>(c1_),
                  static_cast<void*>(q2_), static_cast<void*>(c2_), static_cast<void*>(u2w_),
                  static_cast<void*>(wv_), static_cast<void*>(u1w_), static_cast<void*>(wv1_)})
    if (p) (void)hipFree(p);
}

hipError_t BlocksEngine::ensure_window(const TilePlan& t, int N, hipStream_t s) {
  if (t.q.lo == win_lo_ && t.q.hi == win_hi_ && N <= win_n_) return hipSuccess;
  const size_t n = static_cast<size_t>(N) * t.q.size() * wq_ * d_.C1;
  if (n > q2_cap_) return hipErrorInvalidValue;
  ANX_TRY(hipMemsetAsync(q2_, 0, n * sizeof(float), s));
  win_lo_ = t.q.lo;
  win_hi_ = t.q.hi;
  win_n_ = N;
  return hipSuccess;
}

float* BlocksEngine::q2_row_ptr(const TilePlan& t, int n, int r) {
  return q2_ + static_cast<size_t>(n) * q2_image_stride_floats(t) + static_cast<size_t>(r - t.q.lo) * q2_row_floats();
}

hipError_t BlocksEngine::conv1_chunk(const float* xc, int n, const TilePlan& t, hipStream_t s, int c1_img0) {
  RoctxRange rx("anx conv1");
  const ConvSpec& k1 = b1_.conv;
  const hip::OutView c1v{c1_ + static_cast<size_t>(c1_img0) * t.c1.size() * d_.W1 * d_.C1, t.c1.size(), d_.W1, d_.C1,
                         0, 0, 0};
  if (impl_ == Impl::Mfma && wv1_ != nullptr && use_winograd(k_.conv1_algo, n, t.c1.size(), d_.H1)) {
    const hip::Conv1WinoPlan w = hip::make_conv1_wino_plan(n, t.in.size(), d_.W, k1.K, k1.F);
    if (hip::conv1_wino_v_floats(w) > wv1_cap_) return hipErrorInvalidValue;
    return hip::conv1_wino(w, xc, wv1_, u1w_, b1d_, c1v, true, s, k_);
  }
  if (impl_ == Impl::Mfma) {
    const hip::ConvPlan p =
        hip::make_conv_plan(n, t.in.size(), d_.W, d_.C0, k1.K, k1.F, k1.S, k1.groups, k_.force_vec4, k_.force_scalar);
    ANX_TRY(pack1(p));  // prepared by prepare() for the usual launches: a no-op then
    return hip::conv2d_mfma(p, xc, w1p_, koff1_, b1d_, c1v, true, s);
  }
  return hip::conv2d_direct(xc, w1_, b1d_, c1_, n, t.in.size(), d_.W, d_.C0, k1.K, k1.F, k1.S, 0, k1.groups, true,
                            s);
}

hipError_t BlocksEngine::stage1(const float* x, int N, const TilePlan& t, hipStream_t s, int n_lo, int n_hi) {
  if (n_hi < 0) n_hi = N;
  if (N > max_batch_ || n_lo < 0 || n_hi > N) return hipErrorInvalidValue;
  if (t.out.empty()) return hipSuccess;
  // pool1 rows t.p1 are written into the window t.q at p1.lo - q.lo: they must lie inside it
  if (t.p1.lo < t.q.lo || t.p1.hi > t.q.hi) return hipErrorInvalidValue;
  ANX_TRY(ensure_window(t, N, s));
  const size_t in_img = static_cast<size_t>(t.in.size()) * d_.W * d_.C0;
  const size_t q_img = q2_image_stride_floats(t);
  const int chunk = k_.chunk1 > 0 ? std::min(chunk_, k_.chunk1) : chunk_;
  for (int n0 = n_lo; n0 < n_hi; n0 += chunk) {
    const int n = std::min(chunk, n_hi - n0);
    ANX_TRY(conv1_chunk(x + n0 * in_img, n, t, s));
    RoctxRange rx("anx pool1");
    ANX_TRY(hip::maxpool(c1_, n, t.c1.size(), d_.W1, d_.C1, b1_.pool.F, b1_.pool.S,
                         hip::OutView{q2_ + n0 * q_img, t.q.size(), wq_, d_.C1, t.p1.lo - t.q.lo, b2_.conv.P, 0}, s));
  }
  return hipSuccess;
}

// Conv2 (+ReLU) and Pool2(+LRN) of n images; qc: their conv2 input window.
hipError_t BlocksEngine::conv2_chunk(int n, const TilePlan& t, const float* qc, float* yc, hipStream_t s) {
  RoctxRange rx("anx conv2+pool2+lrn");
  const ConvSpec& k2 = b2_.conv;
  const hip::OutView c2v{c2_, t.c2.size(), d_.W2, d_.C2, 0, 0, 0};
  if (impl_ == Impl::Mfma && wv_ != nullptr && use_winograd(k_.conv2_algo, n, t.c2.size(), d_.H2)) {
    const hip::WinoPlan w = hip::make_wino_plan(n, t.q.size(), wq_, d_.C1, k2.K, k2.groups, u2_m_);
    if (hip::wino_v_floats(w) > wv_cap_) return hipErrorInvalidValue;
    ANX_TRY(hip::wino_input(w, qc, wv_, s));
    ANX_TRY(hip::wino_conv2(w, wv_, u2w_, b2d_, c2v, true, s, k_));
  } else if (impl_ == Impl::Mfma) {
    const hip::ConvPlan p =
        hip::make_conv_plan(n, t.q.size(), wq_, d_.C1, k2.K, k2.F, k2.S, k2.groups, k_.force_vec4, k_.force_scalar);
    ANX_TRY(pack2(p));
    ANX_TRY(hip::conv2d_mfma(p, qc, w2p_, koff2_, b2d_, c2v, true, s));
  } else {
    ANX_TRY(hip::conv2d_direct(qc, w2_, b2d_, c2_, n, t.q.size(), wq_, d_.C1, k2.K, k2.F, k2.S, 0, k2.groups, true,
                               s));
  }
  return pool2_chunk(n, t, yc, s);
}

hipError_t BlocksEngine::pool2_chunk(int n, const TilePlan& t, float* yc, hipStream_t s) {
  const LrnSpec& l = b2_.lrn;
  if (b2_.has_lrn) {
    if (impl_ == Impl::Mfma)
      return hip::maxpool_lrn(c2_, yc, n, t.c2.size(), d_.W2, d_.C2, b2_.pool.F, b2_.pool.S, l.N, l.alpha, l.beta,
                              l.k, l.mode, s);
    // oracle path: separate pool and LRN kernels, staged through the conv1 workspace
    ANX_TRY(hip::maxpool_direct(c2_, c1_, n, t.c2.size(), d_.W2, d_.C2, b2_.pool.F, b2_.pool.S, s));
    return hip::lrn_direct(c1_, yc, n, t.out.size(), d_.Wp2, d_.C2, l.N, l.alpha, l.beta, l.k, l.mode, s);
  }
  return hip::maxpool(c2_, n, t.c2.size(), d_.W2, d_.C2, b2_.pool.F, b2_.pool.S,
                      hip::OutView{yc, t.out.size(), d_.Wp2, d_.C2, 0, 0, 0}, s);
}

hipError_t BlocksEngine::stage2(int N, const TilePlan& t, float* y, hipStream_t s, int n_lo, int n_hi) {
  if (n_hi < 0) n_hi = N;
  if (N > max_batch_ || n_lo < 0 || n_hi > N) return hipErrorInvalidValue;
  if (t.out.empty()) return hipSuccess;
  const size_t q_img = q2_image_stride_floats(t);
  const size_t y_img = static_cast<size_t>(t.out.size()) * d_.Wp2 * d_.C2;
  const int chunk = k_.chunk2 > 0 ? std::min(chunk_, k_.chunk2) : chunk_;
  for (int n0 = n_lo; n0 < n_hi; n0 += chunk) {
    const int n = std::min(chunk, n_hi - n0);
    ANX_TRY(conv2_chunk(n, t, q2_ + n0 * q_img, y + n0 * y_img, s));
  }
  return hipSuccess;
}

bool BlocksEngine::fused_pool1(int N, const TilePlan& t) const {
  if (impl_ != Impl::Mfma || !k_.fuse_pool1 || wv_ == nullptr || d_.C1 % 32 || wq_ > 31) return false;
  // the fused kernel's pooling walk is 3x3 / stride 2 (pool_wino_in_kernel); other pool1 shapes take
  // the unfused maxpool + input transform
  if (b1_.pool.F != 3 || b1_.pool.S != 2) return false;
  // every pool1 row of the window (inside the pooled image) is computed by this tile
  const int lo = std::max(t.q.lo, 0), hi = std::min(t.q.hi, d_.Hp1);
  if (lo < t.p1.lo || hi > t.p1.hi) return false;
  // and every Conv2 launch (chunk, or sub-chunk of one) runs Winograd
  const int chunk = std::min(chunk_, k_.chunk1 > 0 ? k_.chunk1 : chunk_);
  for (int n0 = 0; n0 < N; n0 += chunk) {
    const int n = std::min(chunk, N - n0), sub = k_.conv2_sub > 0 ? std::min(n, k_.conv2_sub) : n;
    if (!use_winograd(k_.conv2_algo, sub, t.c2.size(), d_.H2) ||
        !use_winograd(k_.conv2_algo, n - (n - 1) / sub * sub, t.c2.size(), d_.H2))
      return false;
  }
  return true;
}

bool BlocksEngine::conv1_pools(int N, const TilePlan& t) const {
  if (!k_.conv1_pool || k_.conv1_fused == 0 || k_.conv1_sub > 0 || wv1_ == nullptr || !fused_pool1(N, t)) return false;
  // whole images: every conv1 row, every pool1 row
  if (t.c1.lo != 0 || t.c1.hi != d_.H1 || t.p1.lo != 0 || t.p1.hi != d_.Hp1) return false;
  const int chunk = std::min(chunk_, k_.chunk1 > 0 ? k_.chunk1 : chunk_);
  const ConvSpec& k1 = b1_.conv;
  for (int n0 = 0; n0 < N; n0 += chunk) {
    const int n = std::min(chunk, N - n0);
    if (!use_winograd(k_.conv1_algo, n, t.c1.size(), d_.H1)) return false;
    const hip::Conv1WinoPlan w = hip::make_conv1_wino_plan(n, t.in.size(), d_.W, k1.K, k1.F);
    const hip::OutView win{q2_, t.q.size(), wq_, d_.C1, t.p1.lo - t.q.lo, b2_.conv.P, 0};
    if (w.H1 != d_.H1 || !hip::conv1_fused_pool_eligible(w, win, d_.Hp1, d_.Wp1)) return false;
  }
  return true;
}

bool BlocksEngine::conv2_pools(const TilePlan& t) const {
  const LrnSpec& l = b2_.lrn;
  return k_.conv2_pool && u2_m_ == 4 && b2_.has_lrn && l.N == 5 && d_.C2 == 256 && b2_.pool.F == 3 &&
         b2_.pool.S == 2 && t.c2.lo == 0 && t.c2.size() == d_.H2 && t.out.lo == 0 && t.out.size() == d_.Hp2;
}

hipError_t BlocksEngine::tile_forward(const float* x, int N, const TilePlan& t, float* y, hipStream_t s) {
  if (N > max_batch_) return hipErrorInvalidValue;
  if (t.out.empty()) return hipSuccess;
  if (!fused_pool1(N, t)) {
    ANX_TRY(stage1(x, N, t, s));
    return stage2(N, t, y, s);
  }
  if (conv1_pools(N, t)) return tile_forward_conv1_pool(x, N, t, y, s);
  // conv1 -> (pool1 + Winograd input transform) -> Winograd GEMM -> pool2 + LRN per chunk: the conv2
  // window is never materialised (bit-identical to stage1 + stage2)
  const ConvSpec& k2 = b2_.conv;
  const size_t in_img = static_cast<size_t>(t.in.size()) * d_.W * d_.C0;
  const size_t y_img = static_cast<size_t>(t.out.size()) * d_.Wp2 * d_.C2;
  const int chunk = std::min(chunk_, k_.chunk1 > 0 ? k_.chunk1 : chunk_);
  const size_t c1_img = static_cast<size_t>(t.c1.size()) * d_.W1 * d_.C1;
  const size_t c2_img = static_cast<size_t>(t.c2.size()) * d_.W2 * d_.C2;
  for (int n0 = 0; n0 < N; n0 += chunk) {
    const int n = std::min(chunk, N - n0);
    // Conv1 in sub-chunks (Knobs::conv1_sub): each rewrites the same V workspace, which a small
    // sub-chunk keeps inside the Infinity Cache between the transform and the GEMM
    const int s1 = k_.conv1_sub > 0 ? std::min(n, k_.conv1_sub) : n;
    for (int a0 = 0; a0 < n; a0 += s1)
      ANX_TRY(conv1_chunk(x + (n0 + a0) * in_img, std::min(s1, n - a0), t, s, a0));
    RoctxRange rx("anx pool1+conv2+pool2+lrn");
    const int s2 = k_.conv2_sub > 0 ? std::min(n, k_.conv2_sub) : n;
    for (int b0 = 0; b0 < n; b0 += s2) {
      const int m = std::min(s2, n - b0);
      const hip::WinoPlan w = hip::make_wino_plan(m, t.q.size(), wq_, d_.C1, k2.K, k2.groups, u2_m_);
      if (hip::wino_v_floats(w) > wv_cap_) return hipErrorInvalidValue;
      ANX_TRY(hip::wino_pool_input(w, c1_ + b0 * c1_img, t.c1.size(), d_.W1, t.q.lo, d_.Hp1, d_.Wp1, k2.P, t.c1.lo,
                                   wv_, s, b1_.pool.F, b1_.pool.S));
      const hip::OutView c2v{c2_ + b0 * c2_img, t.c2.size(), d_.W2, d_.C2, 0, 0, 0};
      ANX_TRY(hip::wino_conv2(w, wv_, u2w_, b2d_, c2v, true, s, k_));
    }
    ANX_TRY(pool2_chunk(n, t, y + n0 * y_img, s));
  }
  return hipSuccess;
}

// Whole images with pool1 in the one-kernel Conv1: conv1 + pool1 -> the conv2 window (+ the straddling
// windows' partial maxima in c1_) -> merged input transform -> Winograd GEMM -> pool2 + LRN, per chunk.
// The conv1 map never reaches HBM; bit-identical to the path above (max is exact in any order).
hipError_t BlocksEngine::tile_forward_conv1_pool(const float* x, int N, const TilePlan& t, float* y, hipStream_t s) {
  const ConvSpec &k1 = b1_.conv, &k2 = b2_.conv;
  ANX_TRY(ensure_window(t, N, s));  // zero border once; every interior pixel is rewritten per call
  const size_t in_img = static_cast<size_t>(t.in.size()) * d_.W * d_.C0;
  const size_t y_img = static_cast<size_t>(t.out.size()) * d_.Wp2 * d_.C2;
  const size_t q_img = q2_image_stride_floats(t);
  const size_t p1_img = static_cast<size_t>(d_.Hp1) * d_.Wp1 * d_.C1;
  const size_t c2_img = static_cast<size_t>(t.c2.size()) * d_.W2 * d_.C2;
  const int chunk = std::min(chunk_, k_.chunk1 > 0 ? k_.chunk1 : chunk_);
  for (int n0 = 0; n0 < N; n0 += chunk) {
    const int n = std::min(chunk, N - n0);
    {
      RoctxRange rx("anx conv1+pool1");
      const hip::Conv1WinoPlan w1 = hip::make_conv1_wino_plan(n, t.in.size(), d_.W, k1.K, k1.F);
      const hip::OutView win{q2_ + n0 * q_img, t.q.size(), wq_, d_.C1, t.p1.lo - t.q.lo, k2.P, 0};
      ANX_TRY(hip::conv1_fused_pool(w1, x + n0 * in_img, u1w_, b1d_, win, c1_, d_.Hp1, d_.Wp1, true, s, k_.conv1_fused - 1));
    }
    RoctxRange rx("anx conv2+pool2+lrn");
    const hip::Conv1WinoPlan w1 = hip::make_conv1_wino_plan(n, t.in.size(), d_.W, k1.K, k1.F);
    const int s2 = k_.conv2_sub > 0 ? std::min(n, k_.conv2_sub) : n;
    // pool2 in the GEMM: the pooled map [n][Hp2][Wp2][C2] at c2_, the straddling windows' upper parts
    // behind it (2 x 13 x 13 < 27 x 27 pixels per image: inside the conv2 map's workspace)
    const bool pool2 = conv2_pools(t);
    const size_t pimg = static_cast<size_t>(d_.Hp2) * d_.Wp2 * d_.C2;
    float* const p2 = c2_ + static_cast<size_t>(n) * pimg;
    int ty2 = 0, tx2 = 0;
    for (int b0 = 0; b0 < n; b0 += s2) {
      const int m = std::min(s2, n - b0);
      const hip::WinoPlan w = hip::make_wino_plan(m, t.q.size(), wq_, d_.C1, k2.K, k2.groups, u2_m_);
      if (hip::wino_v_floats(w) > wv_cap_) return hipErrorInvalidValue;
      ANX_TRY(hip::wino_window_merge_input(w, q2_ + (n0 + b0) * q_img, c1_ + b0 * p1_img, b0, w1.ty, w1.tx, t.q.lo,
                                           d_.Hp1, d_.Wp1, k2.P, wv_, s, u2_m_ == 4 ? k_.conv2_in_pg : 32));
      if (pool2) {
        ty2 = w.ty;
        tx2 = w.tx;
        ANX_TRY(hip::wino_gemm_conv2_f45_pool(wv_, u2w_, b2d_, c2_ + b0 * pimg, p2 + b0 * pimg, w.P, w.ty, w.tx, w.Ho,
                                              w.Wo, d_.Hp2, d_.Wp2, w.K, true, s, k_.conv2_occ,
                                              k_.conv2_sched != 0));
      } else {
        const hip::OutView c2v{c2_ + b0 * c2_img, t.c2.size(), d_.W2, d_.C2, 0, 0, 0};
        ANX_TRY(hip::wino_conv2(w, wv_, u2w_, b2d_, c2v, true, s, k_));
      }
    }
    if (pool2) {
      const LrnSpec& l = b2_.lrn;
      ANX_TRY(hip::lrn_pooled_merge(c2_, p2, y + n0 * y_img, n, d_.Hp2, d_.Wp2, d_.C2, ty2, tx2, s2, l.N, l.alpha, l.beta,
                                    l.k, l.mode, s, k_.lrn_wgs));
    } else {
      ANX_TRY(pool2_chunk(n, t, y + n0 * y_img, s));
    }
  }
  return hipSuccess;
}

hipError_t BlocksEngine::forward(const float* x, int N, float* y, hipStream_t s) {
  const DecompPlan p = make_plan(d_.H, d_.W, 1, Decomp::Overlap, b1_, b2_);
  return tile_forward(x, N, p.tiles[0], y, s);
}

}  // namespace anx
