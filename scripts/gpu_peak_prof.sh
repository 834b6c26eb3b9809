#!/bin/bash
# f32 MFMA sustained peak (anx_mfmapeak) and a kernel-trace profile of the 1-GPU bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=cuda-mpi-gpu-cluster-programming_amd/bin
{ timeout -k 10 60 $B/anx_mfmapeak --waves 1 && timeout -k 10 60 $B/anx_mfmapeak --waves 2 && \
  timeout -k 10 60 $B/anx_mfmapeak --waves 4; } > gpurun_out/mfmapeak.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/p_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/p_prof.log 2>&1
rc=$?
cat gpurun_out/mfmapeak.log; tail -1 gpurun_out/p_bench.log | cut -c1-300
exit $rc
