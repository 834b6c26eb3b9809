#!/bin/bash
# Lanes 2 / 3 / 4 at 128 images per GPU with the Conv2 auto occupancy cap (alternating arms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_lanes2
for r in 1 2; do
  for l in 2 3 4; do
    timeout -k 10 200 python -u bench.py --lanes $l --steps 200 --warmup 10 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
  done
done
