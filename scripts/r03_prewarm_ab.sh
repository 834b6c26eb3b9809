#!/bin/bash
# The driver's bench shape (20 timed steps, 5 warmups) with 1 s (default) vs 3 s of untimed clock-settle
# steps, alternating arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_prewarm
for r in 1 2 3; do
  for p in 1 3; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-b1 --prewarm-s $p >> $O.bench.jsonl 2>> $O.err || exit $?
  done
done
