#!/bin/bash
# Conv2 GEMM tile 64x64 (2 per CU) vs 64x128 (1 per CU) under free-running lanes: correctness vs arm 0
# (ab_variants), bench at 128 and 64 images with alternating arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_wide
timeout -k 10 300 python -u tools/ab_variants.py --arms "conv2_wide=0|conv2_wide=1" --batch 128 --lanes 1 --rounds 3 > $O.ab.log 2>&1 || exit $?
for b in 128 64; do
  for r in 1 2; do
    for w in 0 1; do
      timeout -k 10 200 python -u bench.py --batch-per-gpu $b --steps 200 --warmup 10 --no-b1 --knob conv2_wide=$w \
        >> $O.bench.jsonl 2>> $O.err || exit $?
    done
  done
done
