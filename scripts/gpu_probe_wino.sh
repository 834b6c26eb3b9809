#!/bin/bash
# A/B of the interleaved output fold in both Winograd GEMMs at 300 images (tools/probe_wino.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

timeout -k 10 300 python tools/probe_wino.py --batch 300 --bits 257,257 > gpurun_out/probe_wino.log 2>&1 && timeout -k 10 300 python tools/probe_wino.py --batch 300 --knob anx_set_fuse_pool1 --bits 0,1,0,1 > gpurun_out/probe_fuse.log 2>&1
rc=$?
grep bits gpurun_out/probe_c1.log gpurun_out/probe_wino.log
exit $rc
