// anx_hipinit — the bare HIP runtime's cold start, without libanx: the part of a fresh process's
// batch-1 time that is not ours (bench.py b1_process_phases_ms.init_bare_hip). Times, from main()
// entry: hipInit, device count, hipSetDevice + hipFree(0) (context creation), a stream, then the first
// upload of 4 KiB by one of three routes (argv[1]):
//   pageable  hipMalloc + hipMemcpy from pageable memory (the runtime's staged copy path)
//   pinned    hipHostMalloc + hipMalloc + hipMemcpyAsync from the pinned buffer
//   kernel    hipHostMalloc (mapped) + hipMalloc + a copy kernel reading host memory over the link
// The reference's V3 pays these steps inside its timed region (v3_cuda_only/src/main_cuda.cpp:30-35:
// cudaMalloc / cudaMemcpy of the first call create the context).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {
double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}
__global__ void copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
}  // namespace

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "pageable";
  const size_t kBytes = argc > 2 ? static_cast<size_t>(std::atol(argv[2])) : 4096;  // upload size (multiple of 16)
  const double t0 = now_ms();
  double t[6];
  int ndev = 0;
  bool ok = hipInit(0) == hipSuccess;
  t[0] = now_ms();
  ok = ok && hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
  t[1] = now_ms();
  ok = ok && hipSetDevice(0) == hipSuccess && hipFree(nullptr) == hipSuccess;
  t[2] = now_ms();
  hipStream_t s = nullptr;
  ok = ok && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
  t[3] = now_ms();
  void* d = nullptr;
  void* hp = nullptr;
  double t_pin = 0;
  std::vector<char> h(kBytes, 1);
  ok = ok && hipMalloc(&d, kBytes) == hipSuccess;
  if (!std::strcmp(mode, "pinned")) {
    ok = ok && hipHostMalloc(&hp, kBytes, hipHostMallocDefault) == hipSuccess;
    t_pin = now_ms();
    if (ok) std::memcpy(hp, h.data(), kBytes);
    ok = ok && hipMemcpyAsync(d, hp, kBytes, hipMemcpyHostToDevice, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  } else if (!std::strcmp(mode, "kernel")) {
    ok = ok && hipHostMalloc(&hp, kBytes, hipHostMallocMapped) == hipSuccess;
    if (ok) std::memcpy(hp, h.data(), kBytes);
    void* dp = nullptr;
    ok = ok && hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess;
    if (ok) copy_kernel<<<1, 256, 0, s>>>(static_cast<const float4*>(dp), static_cast<float4*>(d), kBytes / 16);
    ok = ok && hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  } else {
    ok = ok && hipMemcpy(d, h.data(), kBytes, hipMemcpyHostToDevice) == hipSuccess;
  }
  t[4] = now_ms();
  if (d) (void)hipFree(d);
  if (hp) (void)hipHostFree(hp);
  if (s) (void)hipStreamDestroy(s);
  t[5] = now_ms();
  std::printf("ANX_JSON {\"ok\": %s, \"mode\": \"%s\", \"devices\": %d, \"hip_init_ms\": %.3f, \"device_count_ms\": %.3f, "
              "\"context_ms\": %.3f, \"stream_ms\": %.3f, \"first_upload_ms\": %.3f, \"pin_alloc_ms\": %.3f, "
              "\"bytes\": %zu, \"teardown_ms\": %.3f, \"total_ms\": %.3f}\n",
              ok ? "true" : "false", mode, ndev, t[0] - t0, t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3],
              t_pin > 0 ? t_pin - t[3] : 0.0, kBytes, t[5] - t[4], t[5] - t0);
  return ok ? 0 : 1;
}
