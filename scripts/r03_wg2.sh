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
# throughput at 64 / 128 images per GPU (the V4 / V5 per-GPU shares), lanes 1-3
for b in 64 128; do
  for l in 1 2 3; do
    timeout -k 10 300 python -u bench.py --batch-per-gpu $b --lanes $l --steps 200 --warmup 10 --no-b1 \
      >> gpurun_out/r03_sweep.jsonl 2>> gpurun_out/r03_sweep.err || exit $?
  done
done
