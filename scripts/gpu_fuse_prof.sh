#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ANX_FUSE_POOL1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fu_prof -o run -- python3 tools/sweep_batch.py --batches 300 --rounds 1 --iters 5 > gpurun_out/fu_prof.log 2>&1
