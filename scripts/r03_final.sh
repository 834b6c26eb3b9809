#!/bin/bash
# Round-end check on the final tree: every GPU test, smoke, the driver's bench shape (x2), 200 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_final
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O.tests.log 2>&1 || exit $?
timeout -k 10 120 python -u __graft_entry__.py smoke > $O.smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > $O.bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --no-b1 >> $O.bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-b1 >> $O.bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model full --steps 50 >> $O.bench.log 2>&1 || exit $?
