#!/bin/bash
# Full AlexNet bf16: Conv1 polyphase (default) vs taps8, tests then interleaved bench A/B and a trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_full_alexnet.py > gpurun_out/fc1_tests.log 2>&1 || { tail -30 gpurun_out/fc1_tests.log; exit 1; }
tail -3 gpurun_out/fc1_tests.log
for r in 1 2; do
  for m in taps8 poly; do
    ANX_FULL_CONV1=$m timeout -k 10 300 python bench.py --model full --steps 30 --warmup 5 > gpurun_out/fc1_${m}_$r.log 2>&1 || exit $?
    echo "conv1 $m round $r: $(grep '"metric"' gpurun_out/fc1_${m}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fc1_prof -o run -- python3 bench.py --model full --steps 10 --warmup 3 > gpurun_out/fc1_prof.log 2>&1
