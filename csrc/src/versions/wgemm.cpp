// anx_wgemm: A/B of the fused Winograd GEMMs on synthetic operands, each kernel timed alone.
//
//   anx_wgemm [--images N] [--iters I]
//
// Conv2: the production path (hip::wino_conv2) against wino_gemm_conv2 configurations and ablations
// (no fold / no fold and no DMA refills). Conv1: the production path (polyphase input transform +
// GEMM) against the GEMM alone on the V it leaves behind. Prints one JSON line per arm: median us per
// launch, MFMA TF/s (the GEMM's f32 MFMA work), and the max |difference| against the production output.
#define ANX_WGEMM_ABLATIONS 1
#include "../hip/wino_gemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

namespace {
// ablations (wino_gemm.hpp): 0 full kernel, 3 no fold + no DMA, 32 no epilogue stores
constexpr int kAbl[] = {0, 3, 32};
#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

float* upload_random(size_t n, unsigned seed, float lo, float hi) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> d(lo, hi);
  for (auto& v : h) v = d(g);
  float* p = nullptr;
  CHECK(hipMalloc(&p, n * sizeof(float)));
  CHECK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}
std::vector<float> download(const float* d, size_t n) {
  std::vector<float> h(n);
  CHECK(hipMemcpy(h.data(), d, n * sizeof(float), hipMemcpyDeviceToHost));
  return h;
}
double time_us(const std::function<hipError_t()>& f, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CHECK(f());
  CHECK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int i = 0; i < iters; ++i) {
    CHECK(hipEventRecord(e0));
    CHECK(f());
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1e3f);
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}
double max_abs_diff(const std::vector<float>& a, const std::vector<float>& b, double* ref_max) {
  double m = 0, r = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    m = std::max(m, static_cast<double>(std::fabs(a[i] - b[i])));
    r = std::max(r, static_cast<double>(std::fabs(b[i])));
  }
  *ref_max = r;
  return m;
}
}  // namespace

int main(int argc, char** argv) {
  int images = 300, iters = 20, only = 0, only_cfg = -1, only_abl = -1, occ = 0;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--images")) images = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--iters")) iters = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--conv")) only = std::atoi(argv[i + 1]);  // 1 or 2: that conv only; 4: Conv2 F(4x4,5x5)
    else if (!std::strcmp(argv[i], "--cfg")) only_cfg = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--abl")) only_abl = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--occ")) occ = std::atoi(argv[i + 1]);  // workgroups-per-CU cap
  }
  if (images < 1 || images > 1400 || iters < 1) {
    std::fprintf(stderr, "usage: anx_wgemm [--images 1..1400] [--iters N]\n");
    return 2;
  }
  using namespace anx;
  const Knobs kn = default_knobs();

  // ---- Conv2: 31x31x96 window -> 27x27x256
  if (only != 1 && only != 4) {
    const hip::WinoPlan w = hip::make_wino_plan(images, 31, 31, 96, 256, 1);
    float* V = upload_random(hip::wino_v_floats(w), 1, -1.f, 1.f);
    float* U = upload_random(hip::wino_u_floats(w), 2, -0.05f, 0.05f);
    float* b = upload_random(256, 3, 0.f, 0.1f);
    const size_t ny = static_cast<size_t>(images) * 27 * 27 * 256;
    float *y0 = nullptr, *y1 = nullptr;
    CHECK(hipMalloc(&y0, ny * sizeof(float)));
    CHECK(hipMalloc(&y1, ny * sizeof(float)));
    const double flop = 2.0 * w.P * 49 * 96 * 256;
    const hip::OutView o0{y0, 27, 27, 256, 0, 0, 0};
    const double t_old = time_us([&] { return hip::wino_conv2(w, V, U, b, o0, true, nullptr, kn); }, iters);
    const auto ref = download(y0, ny);
    std::printf("{\"conv\": 2, \"images\": %d, \"arm\": \"production wino_conv2\", \"us\": %.1f, \"tflops\": %.1f}\n",
                images, t_old, flop / t_old * 1e-6);
    for (int cfg = 0; cfg < 6; ++cfg)
      for (int abl : kAbl) {
        if (only_cfg >= 0 && cfg != only_cfg) continue;
        const hip::OutView ov{y1, 27, 27, 256, 0, 0, 0};
        CHECK(hipMemset(y1, 0, ny * sizeof(float)));
        if (hip::wino_gemm_conv2(V, U, b, ov, w.P, w.ty, w.tx, 27, 27, 96, 256, 1, true, nullptr, occ, abl, cfg) ==
            hipErrorInvalidValue)
          continue;  // no such configuration
        const double t = time_us(
            [&] {
              return hip::wino_gemm_conv2(V, U, b, ov, w.P, w.ty, w.tx, 27, 27, 96, 256, 1, true, nullptr, occ, abl, cfg);
            },
            iters);
        double rmax = 0;
        const double d = max_abs_diff(download(y1, ny), ref, &rmax);
        std::printf("{\"conv\": 2, \"images\": %d, \"arm\": \"wino_gemm cfg=%d abl=%d\", \"us\": %.1f, \"tflops\": "
                    "%.1f, \"max_abs_diff\": %.3g, \"ref_max\": %.3g}\n",
                    images, cfg, abl, t, flop / t * 1e-6, d, rmax);
      }
    for (float* p : {V, U, b, y0, y1}) CHECK(hipFree(p));
  }

  // ---- Conv2 as F(4x4,5x5) (--conv 4): a real window and weights through both tile sizes; the 3x3-tile
  // output is the reference of the 4x4-tile arms (both ~1e-6 of the direct sum)
  if (only == 4 || only == 0) {
    const hip::WinoPlan w3 = hip::make_wino_plan(images, 31, 31, 96, 256, 1, 3);
    const hip::WinoPlan w4 = hip::make_wino_plan(images, 31, 31, 96, 256, 1, 4);
    std::vector<float> xh(static_cast<size_t>(images) * 31 * 31 * 96, 0.f);
    std::mt19937 g(7);
    std::uniform_real_distribution<float> dx(0.f, 1.f), dw(-0.02f, 0.02f);
    for (int n = 0; n < images; ++n)
      for (int y = 2; y < 29; ++y)
        for (int x = 2; x < 29; ++x)
          for (int c = 0; c < 96; ++c) xh[((static_cast<size_t>(n) * 31 + y) * 31 + x) * 96 + c] = dx(g);
    std::vector<float> wh(static_cast<size_t>(256) * 96 * 25);
    for (auto& v : wh) v = dw(g);
    std::vector<float> u3, u4;
    hip::wino_transform_weights_host(w3, wh.data(), u3);
    hip::wino_transform_weights_host(w4, wh.data(), u4);
    float *x = nullptr, *U3 = nullptr, *U4 = nullptr, *V3 = nullptr, *V4 = nullptr, *y0 = nullptr, *y1 = nullptr;
    const size_t ny = static_cast<size_t>(images) * 27 * 27 * 256;
    CHECK(hipMalloc(&x, xh.size() * 4));
    CHECK(hipMemcpy(x, xh.data(), xh.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&U3, u3.size() * 4));
    CHECK(hipMemcpy(U3, u3.data(), u3.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&U4, u4.size() * 4));
    CHECK(hipMemcpy(U4, u4.data(), u4.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&V3, hip::wino_v_floats(w3) * 4));
    CHECK(hipMalloc(&V4, hip::wino_v_floats(w4) * 4));
    CHECK(hipMalloc(&y0, ny * 4));
    CHECK(hipMalloc(&y1, ny * 4));
    float* b = upload_random(256, 3, 0.f, 0.1f);
    const hip::OutView o0{y0, 27, 27, 256, 0, 0, 0}, o1{y1, 27, 27, 256, 0, 0, 0};
    const double ti3 = time_us([&] { return hip::wino_input(w3, x, V3, nullptr); }, iters);
    const double ti4 = time_us([&] { return hip::wino_input(w4, x, V4, nullptr); }, iters);
    const double t3 = time_us([&] { return hip::wino_conv2(w3, V3, U3, b, o0, true, nullptr, kn); }, iters);
    const auto ref = download(y0, ny);
    const double f3 = 2.0 * w3.P * 49 * 96 * 256, f4 = 2.0 * w4.P * 64 * 96 * 256;
    std::printf("{\"conv\": 4, \"images\": %d, \"arm\": \"F(3,5) input transform\", \"us\": %.1f}\n", images, ti3);
    std::printf("{\"conv\": 4, \"images\": %d, \"arm\": \"F(4,5) input transform\", \"us\": %.1f}\n", images, ti4);
    std::printf("{\"conv\": 4, \"images\": %d, \"arm\": \"F(3,5) GEMM (production)\", \"us\": %.1f, \"tflops\": %.1f, "
                "\"direct_equiv_tflops\": %.1f}\n",
                images, t3, f3 / t3 * 1e-6, 2.0 * images * 27 * 27 * 256 * 96 * 25 / t3 * 1e-6);
    std::vector<float> y_prod;  // cfg 0 abl 0 (the compiler-scheduled production kernel): bitwise reference
    for (int cfg = 0; cfg < 5; ++cfg)
      for (int abl : {0, 64, 704, 832, 1856, 2880, 3904, 2752, 1, 65, 2, 3, 67, 4, 16, 32}) {
        if (only_cfg >= 0 && cfg != only_cfg) continue;
        if (only_abl >= 0 && abl != only_abl && !(cfg == 0 && abl == 0)) continue;
        CHECK(hipMemset(y1, 0, ny * 4));
        if (hip::wino_gemm_conv2_f45(V4, U4, b, o1, w4.P, w4.ty, w4.tx, 27, 27, 256, true, nullptr, occ, abl, cfg) ==
            hipErrorInvalidValue)
          continue;
        const double t = time_us(
            [&] {
              return hip::wino_gemm_conv2_f45(V4, U4, b, o1, w4.P, w4.ty, w4.tx, 27, 27, 256, true, nullptr, occ, abl, cfg);
            },
            iters);
        double rmax = 0;
        const auto yo = download(y1, ny);
        const double d = max_abs_diff(yo, ref, &rmax);
        if (cfg == 0 && abl == 0) y_prod = yo;
        const bool bitwise = !y_prod.empty() && std::memcmp(yo.data(), y_prod.data(), ny * 4) == 0;
        std::printf("{\"conv\": 4, \"images\": %d, \"arm\": \"F(4,5) GEMM cfg=%d abl=%d\", \"us\": %.1f, \"tflops\": %.1f, "
                    "\"direct_equiv_tflops\": %.1f, \"max_abs_diff_vs_f35\": %.3g, \"ref_max\": %.3g, "
                    "\"bitwise_vs_production\": %s}\n",
                    images, cfg, abl, t, f4 / t * 1e-6, 2.0 * images * 27 * 27 * 256 * 96 * 25 / t * 1e-6, d, rmax,
                    bitwise ? "true" : "false");
      }
    for (float* p : {x, U3, U4, V3, V4, y0, y1, b}) CHECK(hipFree(p));
  }

  // ---- Conv1: 227x227x3 image -> 55x55x96 (polyphase F(3x3,3x3))
  if (only != 2 && only != 4) {
    const hip::Conv1WinoPlan w = hip::make_conv1_wino_plan(images, 227, 227, 96, 11);
    float* x = upload_random(static_cast<size_t>(images) * 227 * 227 * 3, 4, 0.f, 0.1f);
    std::vector<float> wh(static_cast<size_t>(96) * 3 * 11 * 11);
    std::mt19937 g(5);
    std::uniform_real_distribution<float> d(-0.01f, 0.01f);
    for (auto& v : wh) v = d(g);
    std::vector<float> uh;
    hip::conv1_wino_weights_host(96, 11, wh.data(), uh);
    float* U = nullptr;
    CHECK(hipMalloc(&U, uh.size() * sizeof(float)));
    CHECK(hipMemcpy(U, uh.data(), uh.size() * sizeof(float), hipMemcpyHostToDevice));
    float* b = upload_random(96, 6, 0.f, 0.1f);
    float* V = nullptr;
    CHECK(hipMalloc(&V, hip::conv1_wino_v_floats(w) * sizeof(float)));
    const size_t ny = static_cast<size_t>(images) * 55 * 55 * 96;
    float *y0 = nullptr, *y1 = nullptr;
    CHECK(hipMalloc(&y0, ny * sizeof(float)));
    CHECK(hipMalloc(&y1, ny * sizeof(float)));
    const hip::OutView o0{y0, 55, 55, 96, 0, 0, 0}, o1{y1, 55, 55, 96, 0, 0, 0};
    const double flop = 2.0 * w.P * 25 * 48 * 96;
    const double t_old = time_us([&] { return hip::conv1_wino(w, x, V, U, b, o0, true, nullptr, kn); }, iters);
    const auto ref = download(y0, ny);  // V now holds the transform of x
    std::printf("{\"conv\": 1, \"images\": %d, \"arm\": \"production conv1_wino (input transform + GEMM)\", \"us\": %.1f}\n",
                images, t_old);
    for (int cfg = 0; cfg < 4; ++cfg)
      for (int abl : kAbl) {
        if (only_cfg >= 0 && cfg != only_cfg) continue;
        CHECK(hipMemset(y1, 0, ny * sizeof(float)));
        if (hip::wino_gemm_conv1(V, U, b, o1, w.P, w.ty, w.tx, 55, 55, 96, true, nullptr, occ, abl, cfg) ==
            hipErrorInvalidValue)
          continue;  // no such configuration
        const double t = time_us(
            [&] { return hip::wino_gemm_conv1(V, U, b, o1, w.P, w.ty, w.tx, 55, 55, 96, true, nullptr, occ, abl, cfg); },
            iters);
        double rmax = 0;
        const double dd = max_abs_diff(download(y1, ny), ref, &rmax);
        std::printf("{\"conv\": 1, \"images\": %d, \"arm\": \"wino_gemm cfg=%d abl=%d (GEMM only)\", \"us\": %.1f, "
                    "\"tflops\": %.1f, \"max_abs_diff\": %.3g, \"ref_max\": %.3g}\n",
                    images, cfg, abl, t, flop / t * 1e-6, dd, rmax);
      }
    for (float* p : {x, U, b, V, y0, y1}) CHECK(hipFree(p));
  }
  return 0;
}
