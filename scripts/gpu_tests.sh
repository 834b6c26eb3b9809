#!/bin/bash
# All GPU tests (one pytest process).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/tests_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/tests_gpu.log
exit $rc
