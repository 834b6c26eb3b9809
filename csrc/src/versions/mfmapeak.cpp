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

// Random operands: 8 random floats per lane held in registers, cycled through the unrolled loop
// (different bits every MFMA, no memory traffic), one accumulator chain per wave (the dependent
// chain of the Winograd GEMMs) or four. The guide's DVFS note: random data lowers the loaded clock.
template <int NACC>
__global__ void __launch_bounds__(256) peak32_rand(float* out, int iters, float seed) {
  f32x16 c[NACC] = {};
  float r[8];
  unsigned h = (blockIdx.x * 256 + threadIdx.x) * 2654435761u ^ __float_as_uint(seed);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h = h * 1664525u + 1013904223u;
    r[j] = __uint_as_float(0x3f800000u | (h >> 9)) - 1.5f;  // uniform [-0.5, 0.5)
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      c[k % NACC] = __builtin_amdgcn_mfma_f32_32x32x2f32(r[k & 7], r[(k * 3 + 1) & 7], c[k % NACC], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += c[a][e];
  if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// The Conv2 fused GEMM's operand feed without its memory pipeline: a 64x64 workgroup tile of 4 waves
// (32x32 each), BK = 48 slices of A and B rows in LDS (the kernel's swizzled layout), per group of
// 4 MFMAs two ds_read_b128 fragments; PF = the next group's fragments read before this group's MFMAs.
template <bool PF>
__global__ void __launch_bounds__(256, 2) peak32_lds(float* out, int iters, float seed) {
  constexpr int BK = 48, TILE = 64 * BK;
  __shared__ __attribute__((aligned(16))) float lds[2 * TILE];
  unsigned h0 = threadIdx.x * 2654435761u ^ __float_as_uint(seed);
  for (int i = threadIdx.x; i < 2 * TILE; i += 256) {
    h0 = h0 * 1664525u + 1013904223u;
    lds[i] = __uint_as_float(0x3f800000u | (h0 >> 9)) - 1.5f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5, swz = (r >> 2) & 3;
  int rd[BK / 8];
#pragma unroll
  for (int s4 = 0; s4 < BK / 8; ++s4) rd[s4] = 4 * ((h * (BK / 8) + s4) ^ swz);
  const int a_row = (wm * 32 + r) * BK, b_row = TILE + (wn * 32 + r) * BK;
  f32x16 acc = {};
  for (int i = 0; i < iters; ++i) {
    if constexpr (PF) {
      f32x4 af[2], bf[2];
      af[0] = *reinterpret_cast<const f32x4*>(lds + a_row + rd[0]);
      bf[0] = *reinterpret_cast<const f32x4*>(lds + b_row + rd[0]);
#pragma unroll
      for (int s4 = 0; s4 < BK / 8; ++s4) {
        if (s4 + 1 < BK / 8) {
          af[(s4 + 1) & 1] = *reinterpret_cast<const f32x4*>(lds + a_row + rd[s4 + 1]);
          bf[(s4 + 1) & 1] = *reinterpret_cast<const f32x4*>(lds + b_row + rd[s4 + 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s4 & 1][q], bf[s4 & 1][q], acc, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s4 = 0; s4 < BK / 8; ++s4) {
        const f32x4 af = *reinterpret_cast<const f32x4*>(lds + a_row + rd[s4]);
        const f32x4 bf = *reinterpret_cast<const f32x4*>(lds + b_row + rd[s4]);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q], bf[q], acc, 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += acc[e];
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
  const double l0 = run(peak32_lds<false>, grid, iters / 4, 24.0 * 2 * 32 * 32 * 2, out);
  const double l1 = run(peak32_lds<true>, grid, iters / 4, 24.0 * 2 * 32 * 32 * 2, out);
  std::printf("{\"form\": \"v_mfma_f32_32x32x2_f32 fed by ds_read_b128 (Conv2 GEMM layout), scheduler order\", "
              "\"cus\": %d, \"waves_per_simd\": %d, \"tflops\": %.1f}\n", p.multiProcessorCount, waves, l0);
  std::printf("{\"form\": \"v_mfma_f32_32x32x2_f32 fed by ds_read_b128 (Conv2 GEMM layout), prefetch pinned\", "
              "\"cus\": %d, \"waves_per_simd\": %d, \"tflops\": %.1f}\n", p.multiProcessorCount, waves, l1);
  const double r1 = run(peak32_rand<1>, grid, iters, 16.0 * 2 * 32 * 32 * 2, out);
  const double r4 = run(peak32_rand<4>, grid, iters, 16.0 * 2 * 32 * 32 * 2, out);
  std::printf("{\"form\": \"v_mfma_f32_32x32x2_f32 random operands, 1 accumulator chain\", \"cus\": %d, "
              "\"waves_per_simd\": %d, \"tflops\": %.1f}\n", p.multiProcessorCount, waves, r1);
  std::printf("{\"form\": \"v_mfma_f32_32x32x2_f32 random operands, 4 accumulators\", \"cus\": %d, "
              "\"waves_per_simd\": %d, \"tflops\": %.1f}\n", p.multiProcessorCount, waves, r4);
  CHECK(hipFree(out));
  return 0;
}
