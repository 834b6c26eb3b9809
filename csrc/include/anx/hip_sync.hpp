// anx/hip_sync.hpp — the one workgroup barrier of the hand-written kernels.
//
// `__builtin_amdgcn_s_barrier()` alone only aligns the waves: it does not wait for this wave's own LDS
// traffic. A ds_write still in flight when another wave passes the barrier can be read stale, and a
// ds_read still in flight can return bytes another wave (or an LDS-DMA it issues after the barrier)
// has already overwritten. Round 4 shipped exactly that race (LDS writes before a bare barrier in the
// bf16 Conv1 epilogue, commit 52f2708). `__syncthreads()` is not the fix inside LDS-DMA pipelines: its
// fence waits vmcnt(0) and drains every DMA in flight (cdna_hip_programming.md, "Pipelining across
// barriers").
//
// lds_barrier<VM>() is the form every kernel uses: s_waitcnt lgkmcnt(0) — this wave's LDS reads and
// writes retired — plus, with VM >= 0, vmcnt(VM): this wave's vector-memory ops (LDS-DMA pieces
// included) retired down to VM in flight; then s_barrier. The counted vmcnt is what lets DMA span the
// barrier. scripts/lint.sh rejects a bare __builtin_amdgcn_s_barrier anywhere else.
#pragma once
#include <hip/hip_runtime.h>

namespace anx::hip {

template <int VM = -1>
__device__ __forceinline__ void lds_barrier() {
  static_assert(VM >= -1 && VM < 64, "vmcnt is a 6-bit counter");
  if constexpr (VM >= 0)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VM) : "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // lint: the one allowed use
}

}  // namespace anx::hip
