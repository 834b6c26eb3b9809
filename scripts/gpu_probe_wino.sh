#!/bin/bash
# A/B of the interleaved output fold in both Winograd GEMMs at 300 images (tools/probe_wino.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

timeout -k 10 300 python tools/probe_wino.py --batch 300 --bits 257,769,257,769 > gpurun_out/probe_wino.log 2>&1
rc=$?
grep bits gpurun_out/probe_c1.log gpurun_out/probe_wino.log
exit $rc
