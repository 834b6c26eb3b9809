// anx/lrn_math.hpp — the LRN scale of the fast kernels (pool_lrn.hip, conv_bf16.hip).
//
// y = x / (k + a*s)^beta (reference: v3_cuda_only/src/layers_cuda.cu lrnKernel, powf + division).
// powf and the IEEE division expand to ~250 VALU instructions per output, which made the fused
// pool+LRN kernels VALU-bound (74 us per 256-300 images, one wave-instruction per 4 cycles); here it
// is x * exp2(-beta * log2(k + a*s)) on the hardware v_log_f32 / v_exp_f32 (~1 ulp each, argument
// >= k > 0), 4 instructions. The device oracle (naive.hip) keeps powf and the division.
#pragma once
#include <hip/hip_runtime.h>

namespace anx::hip {

__device__ __forceinline__ float lrn_scale(float s, float k, float a, float beta) {
  return __builtin_amdgcn_exp2f(-beta * __builtin_amdgcn_logf(k + a * s));
}

}  // namespace anx::hip
