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
  int images = 300, iters = 20, only = 0, only_cfg = -1, occ = 0;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--images")) images = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--iters")) iters = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--conv")) only = std::atoi(argv[i + 1]);  // 1 or 2: that conv only
    else if (!std::strcmp(argv[i], "--cfg")) only_cfg = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--occ")) occ = std::atoi(argv[i + 1]);  // workgroups-per-CU cap
  }
  if (images < 1 || images > 1400 || iters < 1) {
    std::fprintf(stderr, "usage: anx_wgemm [--images 1..1400] [--iters N]\n");
    return 2;
  }
  using namespace anx;
  const Knobs kn = default_knobs();

  // ---- Conv2: 31x31x96 window -> 27x27x256
  if (only != 1) {
    const hip::WinoPlan w = hip::make_wino_plan(images, 31, 31, 96, 256, 1);
    const hip::WinoPlan w4 = hip::make_wino_plan(images, 31, 31, 96, 256, 1, 4);
    // a real transform pipeline: random window (zero border of 2) and weights, V / U from them
    std::vector<float> xh(static_cast<size_t>(images) * 31 * 31 * 96, 0.f), wh2(static_cast<size_t>(256) * 96 * 25);
    {
      std::mt19937 gx(1);
      std::uniform_real_distribution<float> dx(0.f, 1.f), dw(-0.02f, 0.02f);
      for (int n = 0; n < images; ++n)
        for (int y = 2; y < 29; ++y)
          for (int x0 = 2; x0 < 29; ++x0)
            for (int c = 0; c < 96; ++c) xh[((static_cast<size_t>(n) * 31 + y) * 31 + x0) * 96 + c] = dx(gx);
      for (auto& v : wh2) v = dw(gx);
    }
    float* xw = nullptr;
    CHECK(hipMalloc(&xw, xh.size() * sizeof(float)));
    CHECK(hipMemcpy(xw, xh.data(), xh.size() * sizeof(float), hipMemcpyHostToDevice));
    std::vector<float> u3h, u4h;
    hip::wino_transform_weights_host(w, wh2.data(), u3h);
    hip::wino_transform_weights_host(w4, wh2.data(), u4h);
    float *V = nullptr, *U = nullptr, *V4 = nullptr, *U4 = nullptr;
    CHECK(hipMalloc(&V, hip::wino_v_floats(w) * sizeof(float)));
    CHECK(hipMalloc(&V4, hip::wino_v_floats(w4) * sizeof(float)));
    CHECK(hipMalloc(&U, u3h.size() * sizeof(float)));
    CHECK(hipMalloc(&U4, u4h.size() * sizeof(float)));
    CHECK(hipMemcpy(U, u3h.data(), u3h.size() * sizeof(float), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(U4, u4h.data(), u4h.size() * sizeof(float), hipMemcpyHostToDevice));
    const double t_in3 = time_us([&] { return hip::wino_input(w, xw, V, nullptr); }, iters);
    const double t_in4 = time_us([&] { return hip::wino_input(w4, xw, V4, nullptr); }, iters);
    std::printf("{\"conv\": 2, \"images\": %d, \"arm\": \"input transform F3 / F4\", \"us\": %.1f, \"us4\": %.1f}\n",
                images, t_in3, t_in4);
    float* b = upload_random(256, 3, 0.f, 0.1f);
    const size_t ny = static_cast<size_t>(images) * 27 * 27 * 256;
    float *y0 = nullptr, *y1 = nullptr;
    CHECK(hipMalloc(&y0, ny * sizeof(float)));
    CHECK(hipMalloc(&y1, ny * sizeof(float)));
    const double flop = 2.0 * w.P * 49 * 96 * 256;
    const hip::OutView o0{y0, 27, 27, 256, 0, 0, 0};
    CHECK(hip::wino_input(w, xw, V, nullptr));
    const double t_old = time_us([&] { return hip::wino_conv2(w, V, U, b, o0, true, nullptr, kn); }, iters);
    const auto ref = download(y0, ny);
    std::printf("{\"conv\": 2, \"images\": %d, \"arm\": \"production wino_conv2\", \"us\": %.1f, \"tflops\": %.1f}\n",
                images, t_old, flop / t_old * 1e-6);
    for (int cfg = 0; cfg < 5; ++cfg)
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
    const double flop4 = 2.0 * w4.P * 64 * 96 * 256;
    for (int cfg = 0; cfg < 3; ++cfg)
      for (int abl : kAbl) {
        if (only_cfg >= 0 && cfg != only_cfg) continue;
        const hip::OutView ov{y1, 27, 27, 256, 0, 0, 0};
        CHECK(hipMemset(y1, 0, ny * sizeof(float)));
        if (hip::wino4_gemm_conv2(V4, U4, b, ov, w4.P, w4.ty, w4.tx, 27, 27, 96, 256, true, nullptr, occ, abl, cfg) ==
            hipErrorInvalidValue)
          continue;
        const double t = time_us(
            [&] {
              return hip::wino4_gemm_conv2(V4, U4, b, ov, w4.P, w4.ty, w4.tx, 27, 27, 96, 256, true, nullptr, occ, abl,
                                           cfg);
            },
            iters);
        double rmax = 0;
        const double d = max_abs_diff(download(y1, ny), ref, &rmax);
        std::printf("{\"conv\": 2, \"images\": %d, \"arm\": \"F4 gemm16 cfg=%d abl=%d\", \"us\": %.1f, \"tflops\": "
                    "%.1f, \"direct3_equiv_tflops\": %.1f, \"max_abs_diff\": %.3g, \"ref_max\": %.3g}\n",
                    images, cfg, abl, t, flop4 / t * 1e-6, flop / t * 1e-6, d, rmax);
      }
    for (float* p : {V, U, V4, U4, xw, b, y0, y1}) CHECK(hipFree(p));
  }

  // ---- Conv1: 227x227x3 image -> 55x55x96 (polyphase F(3x3,3x3))
  if (only != 2) {
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
    // F(4x4,3x3): the whole conv (transform + GEMM) and the GEMM alone per configuration
    {
      const hip::Conv1WinoPlan w4 = hip::make_conv1_wino_plan(images, 227, 227, 96, 11, 4);
      std::vector<float> u4h;
      hip::conv1_wino_weights_host(96, 11, wh.data(), u4h, 4);
      float *U4 = nullptr, *V4 = nullptr;
      CHECK(hipMalloc(&U4, u4h.size() * sizeof(float)));
      CHECK(hipMemcpy(U4, u4h.data(), u4h.size() * sizeof(float), hipMemcpyHostToDevice));
      CHECK(hipMalloc(&V4, hip::conv1_wino_v_floats(w4) * sizeof(float)));
      CHECK(hipMemset(y1, 0, ny * sizeof(float)));
      const double t4 = time_us([&] { return hip::conv1_wino(w4, x, V4, U4, b, o1, true, nullptr, kn); }, iters);
      double rmax = 0;
      const double dd = max_abs_diff(download(y1, ny), ref, &rmax);
      std::printf("{\"conv\": 1, \"images\": %d, \"arm\": \"F4 conv1_wino (input transform + GEMM)\", \"us\": %.1f, "
                  "\"max_abs_diff\": %.3g, \"ref_max\": %.3g}\n",
                  images, t4, dd, rmax);
      const double flop4 = 2.0 * w4.P * 36 * 48 * 96;
      for (int cfg = 0; cfg < 3; ++cfg)
        for (int abl : kAbl) {
          if (only_cfg >= 0 && cfg != only_cfg) continue;
          CHECK(hipMemset(y1, 0, ny * sizeof(float)));
          if (hip::wino4_gemm_conv1(V4, U4, b, o1, w4.P, w4.ty, w4.tx, 55, 55, 96, true, nullptr, occ, abl, cfg) ==
              hipErrorInvalidValue)
            continue;
          const double t = time_us(
              [&] {
                return hip::wino4_gemm_conv1(V4, U4, b, o1, w4.P, w4.ty, w4.tx, 55, 55, 96, true, nullptr, occ, abl, cfg);
              },
              iters);
          const double d4 = max_abs_diff(download(y1, ny), ref, &rmax);
          std::printf("{\"conv\": 1, \"images\": %d, \"arm\": \"F4 gemm16 cfg=%d abl=%d (GEMM only)\", \"us\": %.1f, "
                      "\"tflops\": %.1f, \"max_abs_diff\": %.3g, \"ref_max\": %.3g}\n",
                      images, cfg, abl, t, flop4 / t * 1e-6, d4, rmax);
        }
      CHECK(hipFree(U4));
      CHECK(hipFree(V4));
    }
    for (float* p : {x, U, b, V, y0, y1}) CHECK(hipFree(p));
  }
  return 0;
}
