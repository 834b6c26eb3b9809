#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu_all.log
exit $rc
