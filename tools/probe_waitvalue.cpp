// Probe: do hipStreamWriteValue32 / hipStreamWaitValue32 order work across streams and across
// processes sharing one GPU (the peer transport's device-side flags, anx/schedule.hpp)?
//
//   probe_waitvalue            runs every case, prints one line per case: PASS / FAIL / ERR <what>
// Cases: flag memory from hipMalloc / hipExtMallocWithFlags(hipMallocFinegrained) / signal memory;
// producer in the same process (another stream) and in a forked process (IPC-mapped flag + data).
// Every wait is bounded: the consumer polls its stream for at most 5 s, then releases the wait
// itself with a host copy on a third stream and reports FAIL.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr int kN = 1 << 20;

#define OK(e)                                                                                   \
  do {                                                                                          \
    hipError_t _e = (e);                                                                        \
    if (_e != hipSuccess) {                                                                     \
      std::printf("ERR %s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(_e));        \
      std::fflush(stdout);                                                                      \
      return false;                                                                             \
    }                                                                                           \
  } while (0)

__global__ void copy_k(const float* a, float* b, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void fill_k(float* a, float v, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = v + i;
}
// ~ms milliseconds of busy time (wall clock at 100 MHz), then fill
__global__ void slow_fill_k(float* a, float v, int n, long ticks) {
  const long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = v + i;
}

bool alloc_flag(int kind, unsigned** f) {
  void* p = nullptr;
  if (kind == 0) OK(hipMalloc(&p, 64));
  else if (kind == 1) OK(hipExtMallocWithFlags(&p, 64, hipDeviceMallocFinegrained));
  else OK(hipExtMallocWithFlags(&p, 64, hipMallocSignalMemory));
  OK(hipMemset(p, 0, 64));
  *f = static_cast<unsigned*>(p);
  return true;
}

// consumer side: wait flag >= 1 on s, then copy data -> out; bounded poll
bool consume(unsigned* flag, const float* data, float* out, float v, const char* name) {
  hipStream_t s, rel;
  OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  OK(hipStreamCreateWithFlags(&rel, hipStreamNonBlocking));
  OK(hipStreamWaitValue32(s, flag, 1, hipStreamWaitValueGte, 0xffffffffu));
  copy_k<<<256, 256, 0, s>>>(data, out, kN);
  OK(hipGetLastError());
  const auto t0 = std::chrono::steady_clock::now();
  bool early = hipStreamQuery(s) == hipSuccess;  // must still be blocked right after enqueue
  bool done = false;
  double ms = 0;
  while (!done) {
    done = hipStreamQuery(s) == hipSuccess;
    ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > 5000) break;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  if (!done) {
    const unsigned one = 1;
    OK(hipMemcpyAsync(flag, &one, 4, hipMemcpyHostToDevice, rel));
    OK(hipStreamSynchronize(rel));
  }
  OK(hipStreamSynchronize(s));
  std::vector<float> h(kN);
  OK(hipMemcpy(h.data(), out, kN * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < kN; ++i) bad += h[i] != v + static_cast<float>(i);
  std::printf("%s %s: blocked_at_enqueue=%d released_after_ms=%.1f bad=%d\n",
              done && !early && bad == 0 ? "PASS" : "FAIL", name, !early, ms, bad);
  std::fflush(stdout);
  OK(hipStreamDestroy(s));
  OK(hipStreamDestroy(rel));
  return true;
}

bool same_process(int kind) {
  unsigned* flag;
  if (!alloc_flag(kind, &flag)) return false;
  float *data, *out;
  OK(hipMalloc(&data, kN * 4));
  OK(hipMalloc(&out, kN * 4));
  hipStream_t p;
  OK(hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
  // producer: 200 ms busy kernel that fills data, then the flag write (after it in stream order)
  slow_fill_k<<<256, 256, 0, p>>>(data, 3.f, kN, 20000000L);
  OK(hipGetLastError());
  OK(hipStreamWriteValue32(p, flag, 1, 0));
  char name[64];
  std::snprintf(name, sizeof name, "same-process kind=%d", kind);
  const bool r = consume(flag, data, out, 3.f, name);
  OK(hipStreamSynchronize(p));
  OK(hipStreamDestroy(p));
  OK(hipFree(data));
  OK(hipFree(out));
  OK(hipFree(flag));
  return r;
}

// Fork BEFORE any HIP call: the child is the consumer (owns flag + data, exports IPC handles), the
// parent the producer (fills the child's data through IPC, then writes the child's flag).
int cross_process(int kind) {
  int fds[2], back[2];
  if (pipe(fds) || pipe(back)) return 1;
  const pid_t pid = fork();
  if (pid == 0) {
    close(fds[0]);
    close(back[1]);
    auto child = [&]() -> bool {
      unsigned* flag;
      if (!alloc_flag(kind, &flag)) return false;
      float *data, *out;
      OK(hipMalloc(&data, kN * 4));
      OK(hipMalloc(&out, kN * 4));
      OK(hipMemset(data, 0, kN * 4));
      OK(hipDeviceSynchronize());
      hipIpcMemHandle_t h[2];
      OK(hipIpcGetMemHandle(&h[0], flag));
      OK(hipIpcGetMemHandle(&h[1], data));
      if (write(fds[1], h, sizeof h) != sizeof h) return false;
      char name[64];
      std::snprintf(name, sizeof name, "cross-process kind=%d", kind);
      const bool r = consume(flag, data, out, 5.f, name);
      char c = 0;
      if (read(back[0], &c, 1) != 1) return false;  // producer done (unmapped)
      OK(hipFree(data));
      OK(hipFree(out));
      OK(hipFree(flag));
      return r;
    };
    const bool ok = child();
    if (!ok) {
      // the handle may never have been sent: unblock the parent
      hipIpcMemHandle_t z[2];
      std::memset(z, 0, sizeof z);
      (void)!write(fds[1], z, sizeof z);
    }
    std::fflush(stdout);
    _exit(ok ? 0 : 1);
  }
  close(fds[1]);
  close(back[0]);
  auto parent = [&]() -> bool {
    hipIpcMemHandle_t h[2];
    if (read(fds[0], h, sizeof h) != sizeof h) return false;
    hipIpcMemHandle_t z;
    std::memset(&z, 0, sizeof z);
    if (std::memcmp(&h[0], &z, sizeof z) == 0) return false;
    void *flag, *data;
    OK(hipIpcOpenMemHandle(&flag, h[0], hipIpcMemLazyEnablePeerAccess));
    OK(hipIpcOpenMemHandle(&data, h[1], hipIpcMemLazyEnablePeerAccess));
    hipStream_t p;
    OK(hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
    slow_fill_k<<<256, 256, 0, p>>>(static_cast<float*>(data), 5.f, kN, 20000000L);
    OK(hipGetLastError());
    OK(hipStreamWriteValue32(p, flag, 1, 0));
    OK(hipStreamSynchronize(p));
    OK(hipStreamDestroy(p));
    OK(hipIpcCloseMemHandle(flag));
    OK(hipIpcCloseMemHandle(data));
    return true;
  };
  const bool ok = parent();
  const char c = 1;
  (void)!write(back[1], &c, 1);
  int st = 0;
  waitpid(pid, &st, 0);
  std::printf("cross-process kind=%d producer=%s consumer_exit=%d\n", kind, ok ? "ok" : "failed",
              WIFEXITED(st) ? WEXITSTATUS(st) : -1);
  std::fflush(stdout);
  return 0;
}

}  // namespace

int main() {
  // the forked cases first: the parent must not have touched HIP when it forks
  for (int kind = 0; kind < 3; ++kind) {
    const pid_t pid = fork();  // each case in its own process tree, so a failure cannot leak state
    if (pid == 0) _exit(cross_process(kind));
    int st = 0;
    waitpid(pid, &st, 0);
  }
  int attr = -1;
  if (hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0) == hipSuccess)
    std::printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", attr);
  for (int kind = 0; kind < 3; ++kind) same_process(kind);
  return 0;
}
