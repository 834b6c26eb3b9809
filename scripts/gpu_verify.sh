#!/bin/bash
# Quick re-verification of a fresh tree: all GPU tests, smoke, 1-GPU headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/v_pytest.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/v_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/v_bench.log 2>&1
rc=$?
tail -3 gpurun_out/v_pytest.log; tail -1 gpurun_out/v_smoke.log; tail -1 gpurun_out/v_bench.log | cut -c1-250
exit $rc
