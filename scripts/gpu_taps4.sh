#!/bin/bash
# conv1 scalar gather (variant 1) vs taps4 16-B gathers (variants 9/10): A/B in one process + GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_variants.py --arms="-1:1:2:5,9:-1:2:5,10:-1:2:5" --batch 128 > gpurun_out/abt128.log 2>&1 && \
timeout -k 10 300 python tools/ab_variants.py --arms="-1:3:2:5,-1:-1:2:5" --batch 1 > gpurun_out/abt1.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_taps4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_taps4 -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_taps4.log 2>&1
rc=$?
cat gpurun_out/abt128.log gpurun_out/abt1.log | grep arm; tail -3 gpurun_out/pytest_taps4.log; tail -1 gpurun_out/prof_taps4.log
exit $rc
