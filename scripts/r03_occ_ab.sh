#!/bin/bash
# GEMM occupancy caps under free-running lanes (latest arms: conv1_occ 0 vs 3 with the joint lane start):
# bench step at 128 and 64 images, alternating arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_occ
for b in 128 64; do
  for r in 1 2; do
    for arm in "0 -1" "3 -1"; do
      set -- $arm
      timeout -k 10 200 python -u bench.py --batch-per-gpu $b --steps 200 --warmup 10 --no-b1 --knob conv1_occ=$1 --knob conv2_occ=$2 \
        >> $O.bench.jsonl 2>> $O.err || exit $?
    done
  done
done
