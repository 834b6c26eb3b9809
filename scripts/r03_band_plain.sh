#!/bin/bash
# Band form of the plain Conv2 input transform (the V5 stage split and the unfused path): engine,
# numerics, V4/V5 runtime GPU tests, then the native V5 workload at N=1 (stage split every step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_bp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_winograd_numerics_gpu.py tests/test_v5_runtime.py \
  tests/test_native_cli.py -m gpu -x -q --timeout 120 --timeout-method thread > $O.tests.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload v5 --steps 20 --warmup 3 --no-b1 > $O.v5.log 2>&1 || exit $?
