#!/bin/bash
# The driver's bench shape (20 timed steps after 5 warmups) vs 200 timed steps, alternating, same box:
# how much of the short run is pipeline fill (the lanes restart staggered after each device sync).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_steps
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
done
