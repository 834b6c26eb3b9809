#!/bin/bash
# Fused pool1 + Winograd input transform: bitwise test vs the unfused pair, A/B at 300 images, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -k "fused_pool1 or golden or oracle or tiles" --timeout 120 --timeout-method thread > gpurun_out/fuse_pytest.log 2>&1 && \
timeout -k 10 300 python tools/probe_wino.py --batch 300 --knob anx_set_fuse_pool1 --bits 0,1,0,1 > gpurun_out/probe_fuse.log 2>&1 && \
ANX_FUSE_POOL1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fu_prof -o run -- python3 tools/sweep_batch.py --batches 300 --rounds 1 --iters 5 > gpurun_out/fu_prof.log 2>&1
rc=$?
tail -3 gpurun_out/fuse_pytest.log; grep bits gpurun_out/probe_fuse.log
exit $rc
