#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_versions_gpu.py -x -q -m gpu > gpurun_out/pytest_versions.log 2>&1 && \
timeout -k 10 300 python tools/sweep_batch.py > gpurun_out/sweep_mfma.log 2>&1 && \
timeout -k 10 300 python tools/sweep_batch.py --impl direct --batches 1,8,32 --rounds 2 --iters 2 > gpurun_out/sweep_direct.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_versions.log; cat gpurun_out/sweep_mfma.log gpurun_out/sweep_direct.log 2>/dev/null | grep batch
exit $rc
