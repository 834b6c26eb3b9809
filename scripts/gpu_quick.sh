#!/bin/bash
# quick perf iteration: GPU engine tests + batch sweep (+ optional profile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/sweep_batch.py --batches 1,8,32,64,128,256 > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/sweep_batch.py --batches 128 --rounds 1 --iters 5 > gpurun_out/prof.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; cat gpurun_out/sweep.log
exit $rc
