#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python tools/ab_variants.py --arms="${ARMS:--1:-1:2:0,-1:-1:2:1,-1:-1:2:2,-1:-1:2:3,-1:-1:3:0}" --batch 128 > gpurun_out/ab128.log 2>&1 && \
timeout -k 10 600 python tools/ab_variants.py --arms="${ARMS:--1:-1:2:0,-1:-1:2:1,-1:-1:2:2,-1:-1:2:3,-1:-1:3:0}" --batch 64 > gpurun_out/ab64.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; cat gpurun_out/ab128.log gpurun_out/ab64.log
exit $rc
