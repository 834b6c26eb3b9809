#!/bin/bash
# Staged-version matrix on one MI355X (V1, V2.1/V2.2 x np{1,2,4}, V3, V4 x np{1,2,4}, V5 np1) at
# batch 1 and batch 256, then a kernel trace of the default bench.py step (600 images, 2 lanes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 bash scripts/run_matrix.sh --no-build --batch 1 --iters 3 > gpurun_out/matrix_b1.log 2>&1 && \
timeout -k 10 600 bash scripts/run_matrix.sh --no-build --batch 256 --iters 1 > gpurun_out/matrix_b256.log 2>&1
rc=$?
cp -r logs gpurun_out/matrix_logs 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bench_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench_prof.log 2>&1
