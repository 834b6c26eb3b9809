#!/bin/bash
# Full AlexNet bf16: wave-per-pixel pool2+LRN (default) vs the LDS-tile kernel: tests, A/B, trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_full_alexnet.py > gpurun_out/fl_tests.log 2>&1 || { tail -30 gpurun_out/fl_tests.log; exit 1; }
tail -3 gpurun_out/fl_tests.log
for r in 1 2; do
  for t in 1 0; do
    ANX_BF16_LRN_TILE=$t timeout -k 10 300 python bench.py --model full --steps 30 --warmup 5 > gpurun_out/fl_${t}_$r.log 2>&1 || exit $?
    echo "lrn tile $t round $r: $(grep '"metric"' gpurun_out/fl_${t}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fl_prof -o run -- python3 bench.py --model full --steps 10 --warmup 3 > gpurun_out/fl_prof.log 2>&1
