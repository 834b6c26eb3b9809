#!/bin/bash
# Round 3: native V4 / V5 runtimes + bench JSON semantics on one MI355X.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_v5_runtime.py \
  tests/test_bench_gpu.py "tests/test_full_alexnet.py::test_full_alexnet_rejects_bad_buffers" \
  > gpurun_out/r03_v4_tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc  # a test failure (1) still lets the benches run; anything else stops here
for c in 0 4 8 16; do
  timeout -k 10 300 python -u bench.py --workload v4 --steps 20 --warmup 5 --no-b1 --chunks $c >> gpurun_out/r03_v4_bench.log 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_dp_bench.log 2>&1
