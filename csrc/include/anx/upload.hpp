// anx/upload.hpp — host -> device uploads through one pinned staging buffer.
//
// A process's first hipMemcpy from PAGEABLE memory pays the runtime's staged-copy set-up: 9-10 ms on an
// MI355X box against 0.14 ms for the same 4 KiB from a pinned buffer (anx_hipinit pageable / pinned,
// profiles/r06_cold/). That set-up was half of a fresh batch-1 engine's construction (BlocksEngine: 19.5
// ms, the first of its weight uploads 9-16 ms under the HIP API trace) and the unexplained extra ~8 ms of
// the first engine in a process. Every weight / table upload of the engines goes
// through upload_h2d instead: the bytes are copied into a process-wide pinned buffer (grown on demand,
// kept for the next engine) and DMA'd from there, so no pageable copy path is ever initialised by an
// engine. Thread-safe (one mutex around the shared buffer).
//
// A copy from pinned memory still brings the SDMA queue up on first use (~8 ms for >= 64 KiB); the V3
// CLI, a one-image latency process, therefore also runs with HSA_ENABLE_SDMA=0 (blit-kernel copies):
// 2.5 MiB then take 1.8 ms from a cold process, pinning included.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace anx {

// Synchronous: returns once `bytes` from `src` are in device memory `dst` (or the error). The copies run
// on the stream set by set_upload_stream (default: the null stream, whose first use in a process
// creates its hardware queue; the V3 CLI passes the stream it already has).
hipError_t upload_h2d(void* dst, const void* src, size_t bytes);
void set_upload_stream(hipStream_t s);

}  // namespace anx
