#!/bin/bash
# Round 3: the native V5 runtime on one MI355X — GPU tests (shared-GPU peer ranks, poison, flags /
# notes ordering), then the bench's v5 workload through the C ABI at 1 GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 180 --timeout-method thread -m gpu \
  tests/test_v5_runtime.py > gpurun_out/r03_v5_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload v5 --steps 20 --warmup 5 --no-b1 > gpurun_out/r03_v5_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload v5 --steps 20 --warmup 5 --no-b1 --batch 256 >> gpurun_out/r03_v5_bench.log 2>&1
