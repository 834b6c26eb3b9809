#!/bin/bash
# Winograd vs direct crossover per conv and batch size (tools/ab_variants.py arms: conv2 algo / conv1 algo).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/algo_sweep.log
for b in 1 2 4 8 16 32 64; do
  timeout -k 10 120 python tools/ab_variants.py --batch $b --rounds 5 --iters 20 \
    --arms="-1:-1:0:7:0:4,-1:-1:1:7:0:4,-1:-1:0:7:1:4,-1:-1:1:7:1:4" >> gpurun_out/algo_sweep.log 2>&1 || exit 1
done
grep arm gpurun_out/algo_sweep.log | cut -c1-120
