// anx_convbench — standalone convolution micro-benchmark + self-check (the successor of the
// reference's prebuilt `conv_test` binary, SURVEY §2.1 N30, whose source is missing: it ran a tiled
// conv and printed "Convolution Test Output (first 10 values)").
//
//   anx_convbench [--layer conv1|conv2|conv3|conv4|conv5|all] [--batch N] [--iters K] [--algo direct|winograd]
//
// For each layer shape (AlexNet conv1..conv5) it times the MFMA implicit-GEMM kernel (and the
// Winograd path for 5x5 stride-1 layers), checks the output against the naive device kernel, and
// prints first values, max |diff|, ms and TFLOP/s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "anx/ops.hpp"
#include "anx/rng.hpp"

using namespace anx;

namespace {
void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    std::exit(1);
  }
}
struct Layer {
  const char* name;
  int H, W, C, K, F, S, P, groups;
};
// AlexNet conv layers at their real input sizes (conv3-5 as in the paper, 13x13).
const Layer kLayers[] = {{"conv1", 227, 227, 3, 96, 11, 4, 0, 1},  {"conv2", 27, 27, 96, 256, 5, 1, 2, 1},
                         {"conv3", 13, 13, 256, 384, 3, 1, 1, 1}, {"conv4", 13, 13, 384, 384, 3, 1, 1, 1},
                         {"conv5", 13, 13, 384, 256, 3, 1, 1, 1}};
}  // namespace

int main(int argc, char** argv) {
  std::string which = "all", algo = "direct";
  int N = 64, iters = 20;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--layer" && i + 1 < argc) which = argv[++i];
    else if (a == "--batch" && i + 1 < argc) N = std::atoi(argv[++i]);
    else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (a == "--algo" && i + 1 < argc) algo = argv[++i];
    else {
      std::fprintf(stderr, "usage: anx_convbench [--layer NAME|all] [--batch N] [--iters K] [--algo direct|winograd]\n");
      return 2;
    }
  }
  hipStream_t s;
  ck(hipStreamCreate(&s), "stream");
  hipEvent_t e0, e1;
  ck(hipEventCreate(&e0), "event");
  ck(hipEventCreate(&e1), "event");
  for (const Layer& L : kLayers) {
    if (which != "all" && which != L.name) continue;
    const int Hp = L.H + 2 * L.P, Wp = L.W + 2 * L.P;
    const int Ho = conv_out_dim(L.H, L.F, L.S, L.P), Wo = conv_out_dim(L.W, L.F, L.S, L.P);
    const size_t nx = static_cast<size_t>(N) * L.H * L.W * L.C, nxp = static_cast<size_t>(N) * Hp * Wp * L.C;
    const size_t nw = static_cast<size_t>(L.K) * (L.C / L.groups) * L.F * L.F, ny = static_cast<size_t>(N) * Ho * Wo * L.K;
    std::vector<float> hx(nx), hxp(nxp, 0.f), hw(nw), hb(L.K);
    for (size_t i = 0; i < nx; ++i) hx[i] = rng::uniform(7, 0, i);
    for (size_t i = 0; i < nw; ++i) hw[i] = rng::uniform(7, 1, i) - 0.5f;
    for (int i = 0; i < L.K; ++i) hb[i] = rng::uniform(7, 2, i) - 0.5f;
    for (int n = 0; n < N; ++n)
      for (int y = 0; y < L.H; ++y)
        std::copy_n(&hx[nhwc(n, y, 0, 0, L.H, L.W, L.C)], static_cast<size_t>(L.W) * L.C,
                    &hxp[nhwc(n, y + L.P, L.P, 0, Hp, Wp, L.C)]);
    float *dx, *dxp, *dw, *db, *dy, *dref;
    ck(hipMalloc(&dx, nx * 4), "malloc");
    ck(hipMalloc(&dxp, nxp * 4), "malloc");
    ck(hipMalloc(&dw, nw * 4), "malloc");
    ck(hipMalloc(&db, L.K * 4), "malloc");
    ck(hipMalloc(&dy, ny * 4), "malloc");
    ck(hipMalloc(&dref, ny * 4), "malloc");
    ck(hipMemcpy(dx, hx.data(), nx * 4, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(dxp, hxp.data(), nxp * 4, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(dw, hw.data(), nw * 4, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(db, hb.data(), L.K * 4, hipMemcpyHostToDevice), "H2D");
    ck(hip::conv2d_direct(dx, dw, db, dref, N, L.H, L.W, L.C, L.K, L.F, L.S, L.P, L.groups, false, s), "direct");
    // fast path
    const bool wino = algo == "winograd" && hip::wino_eligible(L.F, L.S, L.C, L.K, L.groups);
    std::vector<float> pk;
    std::vector<int> ko;
    float *dpk = nullptr, *dv = nullptr;
    int* dko = nullptr;
    hip::ConvPlan p = hip::make_conv_plan(N, Hp, Wp, L.C, L.K, L.F, L.S, L.groups);
    hip::WinoPlan wp{};
    if (wino) {
      wp = hip::make_wino_plan(N, Hp, Wp, L.C, L.K, L.groups);
      std::vector<float> u;
      hip::wino_transform_weights_host(wp, hw.data(), pk);  // U [49][K][C/groups]
      ko.assign(1, 0);
      ck(hipMalloc(&dv, hip::wino_v_floats(wp) * 4), "malloc");
    } else {
      hip::pack_conv_weights_host(p, hw.data(), pk, ko);
    }
    ck(hipMalloc(&dpk, pk.size() * 4), "malloc");
    ck(hipMalloc(&dko, ko.size() * 4), "malloc");
    ck(hipMemcpy(dpk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(dko, ko.data(), ko.size() * 4, hipMemcpyHostToDevice), "H2D");
    auto run = [&]() {
      if (wino) {
        ck(hip::wino_input(wp, dxp, dv, s), "wino_input");
        ck(hip::wino_conv2(wp, dv, dpk, db, hip::OutView{dy, Ho, Wo, L.K, 0, 0, 0}, false, s, default_knobs()),
           "wino_conv2");
      } else {
        ck(hip::conv2d_mfma(p, dxp, dpk, dko, db, hip::OutView{dy, Ho, Wo, L.K, 0, 0, 0}, false, s), "mfma");
      }
    };
    run();
    ck(hipStreamSynchronize(s), "sync");
    ck(hipEventRecord(e0, s), "rec");
    for (int i = 0; i < iters; ++i) run();
    ck(hipEventRecord(e1, s), "rec");
    ck(hipEventSynchronize(e1), "sync");
    float ms = 0;
    ck(hipEventElapsedTime(&ms, e0, e1), "elapsed");
    ms /= iters;
    std::vector<float> y(ny), r(ny);
    ck(hipMemcpy(y.data(), dy, ny * 4, hipMemcpyDeviceToHost), "D2H");
    ck(hipMemcpy(r.data(), dref, ny * 4, hipMemcpyDeviceToHost), "D2H");
    double err = 0, mag = 0;
    for (size_t i = 0; i < ny; ++i) {
      err = std::max(err, static_cast<double>(std::fabs(y[i] - r[i])));
      mag = std::max(mag, static_cast<double>(std::fabs(r[i])));
    }
    const double flop = 2.0 * ny * (L.C / L.groups) * L.F * L.F;
    std::printf("Convolution Test Output (first 10 values) [%s]:", L.name);
    for (int i = 0; i < 10; ++i) std::printf(" %.4f", y[i]);
    std::printf("\n%s N=%d %s: %.4f ms  %.2f TFLOP/s (direct-equivalent)  max|diff| %.3e (rel %.3e) %s\n", L.name, N,
                wino ? "winograd" : "mfma", ms, flop / ms / 1e9, err, err / std::max(mag, 1e-30),
                err / std::max(mag, 1e-30) < 1e-5 ? "OK" : "MISMATCH");
    for (void* q : {static_cast<void*>(dx), static_cast<void*>(dxp), static_cast<void*>(dw), static_cast<void*>(db),
                    static_cast<void*>(dy), static_cast<void*>(dref), static_cast<void*>(dpk),
                    static_cast<void*>(dko), static_cast<void*>(dv)})
      if (q) (void)hipFree(q);
  }
  return 0;
}
