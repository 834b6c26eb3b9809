#!/bin/bash
# Free-running lanes restarted staggered (default) vs together after the timed region's device sync:
# 20- and 200-step bench runs, alternating arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_stagger
for r in 1 2; do
  for k in 20 200; do
    timeout -k 10 200 python -u bench.py --steps $k --warmup 5 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
    timeout -k 10 200 python -u bench.py --steps $k --warmup 5 --no-b1 --no-stagger >> $O.bench.jsonl 2>> $O.err || exit $?
  done
done
