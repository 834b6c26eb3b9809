// Pinned-staging uploads (anx/upload.hpp).
#include "anx/upload.hpp"

#include <algorithm>
#include <cstring>
#include <mutex>

namespace anx {

namespace {
std::mutex g_mu;
hipStream_t g_stream = nullptr;
void* g_buf = nullptr;
size_t g_cap = 0;
constexpr size_t kMinCap = 3u << 20;   // the largest upload of a batch-1 engine (conv2 weights, 2.4 MB) fits
constexpr size_t kPiece = 16u << 20;   // larger uploads go through the buffer in pieces
}  // namespace

void set_upload_stream(hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_mu);
  g_stream = s;
}

hipError_t upload_h2d(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return hipSuccess;
  std::lock_guard<std::mutex> lock(g_mu);
  const size_t want = std::min(std::max(bytes, kMinCap), kPiece);
  if (g_cap < want) {
    if (g_buf) (void)hipHostFree(g_buf);
    g_buf = nullptr;
    g_cap = 0;
    const hipError_t e = hipHostMalloc(&g_buf, want, hipHostMallocDefault);
    if (e != hipSuccess) {  // no pinned memory: the plain copy still works
      g_buf = nullptr;
      return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    }
    g_cap = want;
  }
  for (size_t off = 0; off < bytes; off += g_cap) {
    const size_t n = std::min(g_cap, bytes - off);
    std::memcpy(g_buf, static_cast<const char*>(src) + off, n);
    hipError_t e = hipMemcpyAsync(static_cast<char*>(dst) + off, g_buf, n, hipMemcpyHostToDevice, g_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g_stream);  // the buffer is reused by the next piece
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace anx
