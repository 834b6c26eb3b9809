// anx/trace.hpp — roctx ranges for the native engine and runtime.
//
// The reference has no tracing at all: std::chrono around whole runs (v3_cuda_only/src/main_cuda.cpp:
// 30-35, v4_mpi_cuda/src/main_mpi_cuda.cpp:151-160). Here every layer launch of the Blocks engine and
// every communication phase of the multi-rank versions opens a roctx range, so a
// `rocprofv3 --marker-trace --kernel-trace` timeline segments a step into scatter, halo, compute and
// gather per rank. The roctx library is loaded on first use (dlopen of librocprofiler-sdk-roctx,
// then libroctx64); without it, or with ANX_ROCTX=0, a range costs one predictable branch.
#pragma once

namespace anx {

// push/pop a named range (no-ops when roctx is unavailable)
void roctx_push(const char* name);
void roctx_pop();
bool roctx_enabled();

class RoctxRange {
 public:
  explicit RoctxRange(const char* name) : on_(roctx_enabled()) {
    if (on_) roctx_push(name);
  }
  ~RoctxRange() {
    if (on_) roctx_pop();
  }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;

 private:
  bool on_;
};

}  // namespace anx
