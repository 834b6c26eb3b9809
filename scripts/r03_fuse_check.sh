#!/bin/bash
# Fused pool1 transform after a change: its bitwise tests, a kernel trace of one lane at 128 images
# (pool_wino_in_kernel duration vs the unfused pair), and the bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r03_fc
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -k "fused or band" --timeout 120 --timeout-method thread > $O.tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O.prof -o run -- python3 tools/ab_variants.py --arms "fuse_pool1=0|fuse_pool1=1" \
  --batch 128 --rounds 3 > $O.ab.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
done
