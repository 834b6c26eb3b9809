#!/bin/bash
# F(4x4) Winograd (wino_gemm16.hpp) A/B: GEMM arms alone (anx_wgemm), then the bench step with the
# tile knobs (conv1_tile / conv2_tile = 3 or 4) at 128 images.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=cuda-mpi-gpu-cluster-programming_amd/bin
for n in 64 300; do
  echo "## $n images" >> gpurun_out/r03_f4_wg.jsonl
  timeout -k 10 300 $B/anx_wgemm --images $n --iters 20 >> gpurun_out/r03_f4_wg.jsonl 2>&1 || exit $?
done
for t in "3 3" "3 4" "4 3" "4 4"; do
  set -- $t
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-b1 --knob conv1_tile=$1 --knob conv2_tile=$2 \
    >> gpurun_out/r03_f4_bench.jsonl 2>> gpurun_out/r03_f4_bench.err || exit $?
done
