#!/bin/bash
# Stream lanes: bit-identity tests, then bench.py A/B over --lanes and --graph.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k lanes --timeout 120 --timeout-method thread > gpurun_out/lanes_pytest.log 2>&1 && \
for cfg in "1 0" "2 0" "2 1" "3 0" "1 0" "2 0"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lanes $1 --graph $2 > gpurun_out/lanes_b$1_g$2.log 2>&1 || exit $?
  echo "lanes $1 graph $2: $(tail -1 gpurun_out/lanes_b$1_g$2.log | cut -c100-215)"
done
rc=$?
tail -2 gpurun_out/lanes_pytest.log
exit $rc
