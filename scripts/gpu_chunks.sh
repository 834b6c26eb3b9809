#!/bin/bash
# A/B of per-stage launch chunking at 300 images (tools/ab_chunks.py), then the bench with the env override.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_chunks.py --batch 300 --arms "0:0,60:100,100:100,150:150,75:100,120:100,0:100,60:0,30:50,50:100" > gpurun_out/ab_chunks.log 2>&1
rc=$?
cat gpurun_out/ab_chunks.log | grep chunk1
exit $rc
