// anx_bf16bench — the full-AlexNet bf16 conv layers (conv1 polyphase, conv2-5) at their engine
// shapes: times the 128x128 kernels of conv_bf16.hip (register-staged / LDS-DMA ring) and every
// wide-tile config of conv_bf16_big.hip in interleaved rounds (one process, same device), and
// checks each output against the register-staged kernel (same packed operands, fp32 accumulation:
// only summation order and the final bf16 rounding differ).
//
//   anx_bf16bench [--batch N] [--iters K] [--rounds R] [--layer conv1p|conv2|...|all]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "anx/bf16_ops.hpp"
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
  int Hp, Wp, C, K, F;
};
const Layer kLayers[] = {{"conv1p", 57, 57, 48, 96, 3},
                         {"conv2", 31, 31, 96, 256, 5},
                         {"conv3", 15, 15, 256, 384, 3},
                         {"conv4", 15, 15, 384, 384, 3},
                         {"conv5", 15, 15, 384, 256, 3},
                         {"fc6", 1, 1, 9216, 4096, 1},
                         {"fc7", 1, 1, 4096, 4096, 1},
                         {"fc8", 1, 1, 4096, 1000, 1}};
float bf2f(uint16_t b) {
  const uint32_t u = static_cast<uint32_t>(b) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
}  // namespace

int main(int argc, char** argv) {
  std::string which = "all";
  int N = 256, iters = 20, rounds = 3;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--batch" && i + 1 < argc) N = std::atoi(argv[++i]);
    else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (a == "--rounds" && i + 1 < argc) rounds = std::atoi(argv[++i]);
    else if (a == "--layer" && i + 1 < argc) which = argv[++i];
    else {
      std::fprintf(stderr, "usage: anx_bf16bench [--batch N] [--iters K] [--rounds R] [--layer NAME|all]\n");
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
    const hip::ConvPlanB p = hip::make_conv_plan_bf16(N, L.Hp, L.Wp, L.C, L.K, L.F, 1, 1);
    const size_t nx = static_cast<size_t>(N) * L.Hp * L.Wp * L.C, ny = static_cast<size_t>(N) * p.Ho * p.Wo * L.K;
    const size_t nw = static_cast<size_t>(L.K) * L.C * L.F * L.F;
    std::vector<uint16_t> hx(nx);
    std::vector<float> hw(nw), hb(L.K);
    for (size_t i = 0; i < nx; ++i) hx[i] = hip::f32_to_bf16_bits(2.f * rng::uniform(11, 0, i) - 1.f);
    const float sc = std::sqrt(6.f / (L.C * L.F * L.F));
    for (size_t i = 0; i < nw; ++i) hw[i] = sc * (2.f * rng::uniform(11, 1, i) - 1.f);
    for (int i = 0; i < L.K; ++i) hb[i] = 0.1f * (2.f * rng::uniform(11, 2, i) - 1.f);
    std::vector<uint16_t> pk;
    std::vector<int> ko;
    hip::pack_conv_weights_bf16(p, hw.data(), pk, ko);
    void *dx, *dw, *dy0, *dy1, *dwb = nullptr;
    int* dko;
    float* db;
    ck(hipMalloc(&dx, nx * 2), "malloc");
    ck(hipMalloc(&dw, pk.size() * 2), "malloc");
    ck(hipMalloc(&dko, ko.size() * 4), "malloc");
    ck(hipMalloc(&db, L.K * 4), "malloc");
    ck(hipMalloc(&dy0, ny * 2), "malloc");
    ck(hipMalloc(&dy1, ny * 2), "malloc");
    ck(hipMemcpy(dx, hx.data(), nx * 2, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(dw, pk.data(), pk.size() * 2, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(dko, ko.data(), ko.size() * 4, hipMemcpyHostToDevice), "H2D");
    ck(hipMemcpy(db, hb.data(), L.K * 4, hipMemcpyHostToDevice), "H2D");
    const hip::OutViewB o0{static_cast<__bf16*>(dy0), p.Ho, p.Wo, L.K, 0, 0, 0};
    const hip::OutViewB o1{static_cast<__bf16*>(dy1), p.Ho, p.Wo, L.K, 0, 0, 0};
    // arms: -2 register-staged 128x128 (unsplit), -1 LDS-DMA ring 128x128 (the legacy FC split-K),
    // c = wide-tile config c; FC layers: 100*ks + c = config c with K split ks ways (+ reduce)
    const bool fc = L.Hp == 1;
    std::vector<int> arms = {-2, -1};
    for (int c = 0; c < hip::conv_bf16_big_cfgs(); ++c) {
      if (!hip::conv_bf16_big_ok(p, c, o1)) continue;
      if (!fc) {
        arms.push_back(c);
        continue;
      }
      for (int ks : {1, 2, 4, 8, 16})
        if (ks * 4 <= p.kpad / 64 && ks > 1 && (c == 1 || c == 3 || c >= 5)) arms.push_back(100 * ks + c);
    }
    float* dws = nullptr;
    if (fc) ck(hipMalloc(&dws, static_cast<size_t>(16) * N * L.K * 4), "malloc ws");
    const int ks_legacy = hip::fc_split_k(p);
    auto run = [&](int arm) {
      if (arm == -2) {
        ck(hip::conv2d_bf16(p, dx, dw, dko, db, o0, nullptr, true, s, {}, 0), "conv2d_bf16");
      } else if (arm == -1) {
        if (fc && ks_legacy > 1) {
          ck(hip::conv2d_bf16(p, dx, dw, dko, db, o1, nullptr, true, s, hip::SplitK{ks_legacy, dws}, 2), "legacy split");
          ck(hip::splitk_reduce_bf16(dws, ks_legacy, N, L.K, db, true, o1, nullptr, s), "reduce");
        } else {
          ck(hip::conv2d_bf16(p, dx, dw, dko, db, o1, nullptr, true, s, {}, 2), "conv2d_bf16 glds");
        }
      } else if (arm >= 100) {
        const int ks = arm / 100, c = arm % 100;
        ck(hip::conv2d_bf16_big(p, c, dx, dw, dko, db, o1, true, s, hip::SplitK{ks, dws}), "big split");
        ck(hip::splitk_reduce_bf16(dws, ks, N, L.K, db, true, o1, nullptr, s), "reduce");
      } else {
        ck(hip::conv2d_bf16_big(p, arm, dx, dw, dko, db, o1, true, s), "conv2d_bf16_big");
      }
    };
    if (fc) {
      const hip::BigFc f = hip::pick_bf16_big_fc(p);
      std::printf("%s: legacy ksplit %d, picker cfg %d ksplit %d (arm %d)\n", L.name, ks_legacy, f.cfg, f.ksplit,
                  100 * f.ksplit + f.cfg);
    }
    std::vector<uint16_t> y0(ny), y1(ny);
    run(-2);
    ck(hipMemcpy(y0.data(), dy0, ny * 2, hipMemcpyDeviceToHost), "D2H");
    float mag = 0;
    for (size_t i = 0; i < ny; ++i) mag = std::max(mag, std::fabs(bf2f(y0[i])));
    std::vector<std::vector<float>> ms(arms.size());
    for (size_t a = 0; a < arms.size(); ++a) {
      if (arms[a] == -2) continue;
      ck(hipMemset(dy1, 0xff, ny * 2), "memset");  // NaN fill: unwritten outputs show up
      run(arms[a]);
      ck(hipMemcpy(y1.data(), dy1, ny * 2, hipMemcpyDeviceToHost), "D2H");
      double err = 0;
      size_t bad = 0;
      for (size_t i = 0; i < ny; ++i) {
        const float d = std::fabs(bf2f(y1[i]) - bf2f(y0[i]));
        if (!(d <= 1e-2f * mag)) ++bad;
        if (d > err || d != d) err = d != d ? INFINITY : d;
      }
      std::printf("%s arm %d: max|diff| %.3e of max|y| %.3e, %zu outside 1e-2 %s\n", L.name, arms[a], err, mag, bad,
                  bad ? "MISMATCH" : "OK");
    }
    for (int r = 0; r < rounds; ++r)
      for (size_t a = 0; a < arms.size(); ++a) {
        run(arms[a]);
        ck(hipEventRecord(e0, s), "rec");
        for (int i = 0; i < iters; ++i) run(arms[a]);
        ck(hipEventRecord(e1, s), "rec");
        ck(hipEventSynchronize(e1), "sync");
        float t = 0;
        ck(hipEventElapsedTime(&t, e0, e1), "elapsed");
        ms[a].push_back(t / iters);
      }
    const double flop = 2.0 * ny * L.C * L.F * L.F;
    for (size_t a = 0; a < arms.size(); ++a) {
      std::sort(ms[a].begin(), ms[a].end());
      const double med = ms[a][ms[a].size() / 2];
      std::printf("{\"layer\": \"%s\", \"batch\": %d, \"arm\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"tflops\": %.1f}\n",
                  L.name, N, arms[a], med, ms[a][0], flop / med / 1e9);
    }
    for (void* q : {dx, dw, dwb, static_cast<void*>(dko), static_cast<void*>(db), dy0, dy1, static_cast<void*>(dws)})
      if (q) (void)hipFree(q);
  }
  return 0;
}
