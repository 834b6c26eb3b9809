// Naive HIP kernels: the device-side correctness oracle.
//
// One thread per output element, channel fastest — the same decomposition as the reference's
// convKernel / reluKernel / poolKernel / lrnKernel (v3_cuda_only/src/layers_cuda.cu:20-152,
// v4_mpi_cuda/src/layers_mpi_cuda.cu:25-136), plus batch, groups and both LRN formulas.
// These are deliberately simple: the MFMA path (conv_mfma.hip) is checked against them and
// against PyTorch on the GPU.
#include <hip/hip_runtime.h>

#include <cmath>

#include "anx/ops.hpp"

namespace anx::hip {
namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(size_t n) {
  size_t g = (n + kBlock - 1) / kBlock;
  return static_cast<unsigned>(g > 0x7fffffffu ? 0x7fffffffu : g);
}

__global__ void __launch_bounds__(kBlock) conv_direct_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ b, float* __restrict__ y,
                                                             int N, int H, int W, int C, int K, int F, int S, int P,
                                                             int groups, int Ho, int Wo, int relu) {
  const size_t total = static_cast<size_t>(N) * Ho * Wo * K;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int k = static_cast<int>(i % K);
    size_t r = i / K;
    const int ox = static_cast<int>(r % Wo);
    r /= Wo;
    const int oy = static_cast<int>(r % Ho);
    const int n = static_cast<int>(r / Ho);
    const int Cg = C / groups, Kg = K / groups, g = k / Kg;
    float acc = b ? b[k] : 0.f;
    for (int c = 0; c < Cg; ++c)
      for (int fh = 0; fh < F; ++fh) {
        const int iy = oy * S + fh - P;
        if (iy < 0 || iy >= H) continue;
        for (int fw = 0; fw < F; ++fw) {
          const int ix = ox * S + fw - P;
          if (ix < 0 || ix >= W) continue;
          acc = fmaf(x[nhwc(n, iy, ix, g * Cg + c, H, W, C)], w[((static_cast<size_t>(k) * Cg + c) * F + fh) * F + fw],
                     acc);
        }
      }
    y[i] = relu ? fmaxf(acc, 0.f) : acc;
  }
}

__global__ void __launch_bounds__(kBlock) relu_kernel(float* __restrict__ x, size_t n) {
  // float4 body + scalar tail; x comes from hipMalloc / torch (16-B aligned).
  const size_t n4 = n / 4;
  float4* x4 = reinterpret_cast<float4*>(x);
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n4; i += stride) {
    float4 v = x4[i];
    v.x = fmaxf(v.x, 0.f);
    v.y = fmaxf(v.y, 0.f);
    v.z = fmaxf(v.z, 0.f);
    v.w = fmaxf(v.w, 0.f);
    x4[i] = v;
  }
  for (size_t i = n4 * 4 + blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    x[i] = fmaxf(x[i], 0.f);
}

__global__ void __launch_bounds__(kBlock) pool_direct_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             int N, int H, int W, int C, int F, int S, int Ho,
                                                             int Wo) {
  const size_t total = static_cast<size_t>(N) * Ho * Wo * C;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    size_t r = i / C;
    const int ox = static_cast<int>(r % Wo);
    r /= Wo;
    const int oy = static_cast<int>(r % Ho);
    const int n = static_cast<int>(r / Ho);
    float m = -INFINITY;
    for (int fh = 0; fh < F; ++fh)
      for (int fw = 0; fw < F; ++fw) {
        const int iy = oy * S + fh, ix = ox * S + fw;
        if (iy < H && ix < W) m = fmaxf(m, x[nhwc(n, iy, ix, c, H, W, C)]);
      }
    y[i] = m;
  }
}

__global__ void __launch_bounds__(kBlock) lrn_direct_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                            size_t P, int C, int size, float a, float beta,
                                                            float k) {
  const size_t total = P * C;
  const int half = size / 2;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    const size_t base = i - c;
    float s = 0.f;
    const int lo = c - half < 0 ? 0 : c - half;
    const int hi = c + half >= C ? C - 1 : c + half;
    for (int j = lo; j <= hi; ++j) {
      const float v = x[base + j];
      s = fmaf(v, v, s);
    }
    y[i] = x[i] / powf(k + a * s, beta);
  }
}

__global__ void __launch_bounds__(kBlock) fill_kernel(float* __restrict__ x, size_t n, float v) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    x[i] = v;
}

// Copy with a fixed number of workgroups (the receive-side work of a collective that owns that many
// CUs: RCCL's receive channels copying from their FIFOs into the user buffer). 16-B vectors, grid-stride.
__global__ void __launch_bounds__(kBlock) channel_copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                              size_t n4) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n4;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

}  // namespace

hipError_t channel_copy(void* dst, const void* src, size_t bytes, int workgroups, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if (bytes % 16 || workgroups < 1 || reinterpret_cast<uintptr_t>(dst) % 16 || reinterpret_cast<uintptr_t>(src) % 16)
    return hipErrorInvalidValue;
  channel_copy_kernel<<<static_cast<unsigned>(workgroups), kBlock, 0, s>>>(static_cast<const float4*>(src),
                                                                          static_cast<float4*>(dst), bytes / 16);
  return hipGetLastError();
}

hipError_t conv2d_direct(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C,
                         int K, int F, int S, int P, int groups, bool relu, hipStream_t s) {
  const int Ho = conv_out_dim(H, F, S, P), Wo = conv_out_dim(W, F, S, P);
  const size_t total = static_cast<size_t>(N) * Ho * Wo * K;
  if (total == 0) return hipSuccess;
  conv_direct_kernel<<<grid_for(total), kBlock, 0, s>>>(x, w, b, y, N, H, W, C, K, F, S, P, groups, Ho, Wo,
                                                        relu ? 1 : 0);
  return hipGetLastError();
}

hipError_t relu(float* x, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  size_t g = grid_for(n / 4 + 1);
  if (g > 4096) g = 4096;
  relu_kernel<<<static_cast<unsigned>(g), kBlock, 0, s>>>(x, n);
  return hipGetLastError();
}

hipError_t maxpool_direct(const float* x, float* y, int N, int H, int W, int C, int F, int S, hipStream_t s) {
  const int Ho = pool_out_dim(H, F, S), Wo = pool_out_dim(W, F, S);
  const size_t total = static_cast<size_t>(N) * Ho * Wo * C;
  if (total == 0) return hipSuccess;
  pool_direct_kernel<<<grid_for(total), kBlock, 0, s>>>(x, y, N, H, W, C, F, S, Ho, Wo);
  return hipGetLastError();
}

hipError_t lrn_direct(const float* x, float* y, int N, int H, int W, int C, int size, float alpha, float beta,
                      float k, LrnMode mode, hipStream_t s) {
  const size_t P = static_cast<size_t>(N) * H * W;
  if (P == 0) return hipSuccess;
  const float a = mode == LrnMode::DivN ? alpha / static_cast<float>(size) : alpha;
  lrn_direct_kernel<<<grid_for(P * C), kBlock, 0, s>>>(x, y, P, C, size, a, beta, k);
  return hipGetLastError();
}

hipError_t fill(float* x, size_t n, float v, hipStream_t s) {
  if (n == 0) return hipSuccess;
  size_t g = grid_for(n);
  if (g > 8192) g = 8192;
  fill_kernel<<<static_cast<unsigned>(g), kBlock, 0, s>>>(x, n, v);
  return hipGetLastError();
}

}  // namespace anx::hip
