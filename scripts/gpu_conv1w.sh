#!/bin/bash
# Winograd-conv session: numerics tests, in-process A/B (conv1 direct vs polyphase-Winograd ring
# shapes; conv2 fused-kernel configurations), batch sweep, kernel-trace profile of the bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${BATCH:-300}
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c1w_pytest.log 2>&1 && \
timeout -k 10 300 python tools/ab_variants.py --arms="-1:-1:0:7:2:4,-1:-1:0:15:2:4,-1:-1:0:14:2:4,-1:-1:0:12:2:4" --batch $B > gpurun_out/c1w_ab.log 2>&1 && \
timeout -k 10 300 python tools/sweep_batch.py --batches 128,256,300,302 --rounds 3 --iters 8 > gpurun_out/c1w_sweep.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c1w_prof -o run -- python3 tools/sweep_batch.py --batches $B --rounds 1 --iters 5 > gpurun_out/c1w_prof.log 2>&1
rc=$?
tail -3 gpurun_out/c1w_pytest.log; grep -h arm gpurun_out/c1w_ab.log; grep -h batch gpurun_out/c1w_sweep.log
exit $rc
