#!/bin/bash
# Lane-count sweep at 64 / 128 images per GPU (the V4 / V5 per-GPU shares), then the full bf16 model
# at 256 images with a kernel trace (anx bench, one process per arm).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in 64 128; do
  for l in 2 3 4; do
    timeout -k 10 200 python -u bench.py --batch-per-gpu $b --lanes $l --steps 200 --warmup 10 --no-b1 \
      >> gpurun_out/r03_lanes_sweep.jsonl 2>> gpurun_out/r03_lanes_sweep.err || exit $?
  done
done
timeout -k 10 200 python -u bench.py --model full --steps 50 >> gpurun_out/r03_full_bench.jsonl 2>> gpurun_out/r03_lanes_sweep.err || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_full" -o full -- \
  python -u "$GRAFT_REPO_ROOT/bench.py" --model full --steps 20 --prewarm-s 0.2 >> "$GRAFT_REPO_ROOT/gpurun_out/r03_full_bench.jsonl" 2>> "$GRAFT_REPO_ROOT/gpurun_out/r03_lanes_sweep.err"
