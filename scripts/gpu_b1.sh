#!/bin/bash
# Batch-1 latency (the reference's V3 configuration): native v3 warm timing per algorithm and a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=cuda-mpi-gpu-cluster-programming_amd/bin
{ for c1 in direct; do for c2 in direct; do
    echo "== conv1 $c1 conv2 $c2"
    timeout -k 10 60 $B/anx --version v3 --batch 1 --init const --lrn-alpha-mode raw --iters 200 --conv1-algo $c1 --conv2-algo $c2 || exit 1
  done; done; } > gpurun_out/b1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/b1_prof -o run -- $B/anx --version v3 --batch 1 --iters 50 --conv1-algo direct --conv2-algo direct > gpurun_out/b1_prof.log 2>&1
rc=$?
grep -E "==|ANX_JSON" gpurun_out/b1.log | cut -c1-200
exit $rc
