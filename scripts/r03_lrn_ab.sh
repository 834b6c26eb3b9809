#!/bin/bash
# pool2 + LRN: row-walk kernel vs 2-pixel waves (ANX_LRN_ROWS), bitwise + timing, then the bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r03_lrn
timeout -k 10 200 python -u tools/probe_lrn_rows.py > $O.probe.jsonl 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O.prof -o run -- python3 tools/probe_lrn_rows.py > $O.prof.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
  ANX_LRN_ROWS=1 timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-b1 >> $O.bench.jsonl 2>> $O.err || exit $?
done
