// anx_mfmapeak: sustained f32 matrix-core throughput of this MI355X under a full-chip load, the
// roofline denominator for the Winograd GEMMs (conv1_wino.hip, winograd.hip). Every CU runs
// `--waves` waves per SIMD, each issuing chains of independent MFMAs on register operands (no
// memory traffic inside the loop); hipEvent timing over `--iters` loop trips.
//   anx_mfmapeak [--iters N] [--waves W]    -> one JSON line per instruction form
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace {
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// 32x32x2 f32: 4 independent accumulators per wave (latency 64 cycles = issue 64: one chain would
// already saturate; four remove any doubt)
__global__ void __launch_bounds__(256) peak32(float* out, int iters, float seed) {
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float a = seed + threadIdx.x * 1e-7f, b = seed - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += c0[e] + c1[e] + c2[e] + c3[e];
  if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keeps the chains live
}

__global__ void __launch_bounds__(256) peak16(float* out, int iters, float seed) {
  f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float a = seed + threadIdx.x * 1e-7f, b = seed - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) s += c0[e] + c1[e] + c2[e] + c3[e];
  if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
double run(K kernel, int grid, int iters, double flop_per_wave_iter, float* out) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  kernel<<<grid, 256>>>(out, 16, 1.0f);  // warm-up (clocks, code load)
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  kernel<<<grid, 256>>>(out, iters, 1.0f);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  const double waves = static_cast<double>(grid) * 4;
  return waves * iters * flop_per_wave_iter / (ms * 1e-3) / 1e12;
}
}  // namespace

int main(int argc, char** argv) {
  int iters = 20000, waves = 2;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--iters")) iters = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--waves")) waves = std::atoi(argv[i + 1]);
  }
  if (iters < 1 || waves < 1 || waves > 8) {
    std::fprintf(stderr, "usage: anx_mfmapeak [--iters N>0] [--waves 1..8]\n");
    return 2;
  }
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount * waves;  // 256-thread workgroups: one wave per SIMD each
  float* out = nullptr;
  CHECK(hipMalloc(&out, static_cast<size_t>(grid) * 256 * sizeof(float)));
  // flop per wave per loop trip: 16 MFMAs x (2 * M * N * K)
  const double t32 = run(peak32, grid, iters, 16.0 * 2 * 32 * 32 * 2, out);
  const double t16 = run(peak16, grid, iters, 32.0 * 2 * 16 * 16 * 4, out);
  std::printf("{\"form\": \"v_mfma_f32_32x32x2_f32\", \"cus\": %d, \"waves_per_simd\": %d, \"tflops\": %.1f}\n",
              p.multiProcessorCount, waves, t32);
  std::printf("{\"form\": \"v_mfma_f32_16x16x4_f32\", \"cus\": %d, \"waves_per_simd\": %d, \"tflops\": %.1f}\n",
              p.multiProcessorCount, waves, t16);
  CHECK(hipFree(out));
  return 0;
}
