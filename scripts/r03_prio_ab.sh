#!/bin/bash
# Side-lane stream priority under free-running lanes (bench --lane-priority 0 / -1), alternating arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_prio
for r in 1 2; do
  for p in 0 -1; do
    timeout -k 10 200 python -u bench.py --lane-priority $p --steps 200 --warmup 10 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
  done
done
