#!/bin/bash
# A/B of the register-staged vs LDS-DMA fused Winograd kernel, numerics vs arm 0, plus a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_variants.py --arms="-1:-1:2:1,-1:-1:2:5" --batch 128 > gpurun_out/abg128.log 2>&1 && \
timeout -k 10 300 python tools/ab_variants.py --arms="-1:-1:2:1,-1:-1:2:5" --batch 64 > gpurun_out/abg64.log 2>&1 && \
ANX_WINO_FUSED_CFG=5 timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -m gpu > gpurun_out/pytest_glds.log 2>&1 && \
ANX_WINO_FUSED_CFG=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_glds -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_glds.log 2>&1
rc=$?
cat gpurun_out/abg128.log gpurun_out/abg64.log; tail -3 gpurun_out/pytest_glds.log; tail -1 gpurun_out/prof_glds.log
exit $rc
