#!/bin/bash
# GEMM configuration / epilogue A/B (anx_wgemm) at 64 and 300 images, each kernel alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=cuda-mpi-gpu-cluster-programming_amd/bin
for n in 64 300; do
  echo "## $n images" >> gpurun_out/r03_wg2.jsonl
  timeout -k 10 240 $B/anx_wgemm --images $n --iters 20 >> gpurun_out/r03_wg2.jsonl 2>&1 || exit $?
done
