#!/bin/bash
# Round 3: standalone per-kernel HBM bytes (FETCH_SIZE / WRITE_SIZE, one pass each), clock and MFMA
# busy of the bench step at 128 images on one lane (counter passes serialise dispatches), then the
# V5 halo pipeline on ranks sharing the GPU (chunks 1 vs auto).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH="bench.py --lanes 1 --steps 6 --warmup 2 --no-b1 --prewarm-s 0"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace \
  --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 $BENCH > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d gpurun_out/pmc_write -o run -- python3 $BENCH > gpurun_out/pmc_write.log 2>&1 &&
python3 tools/pmc_clock.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/r03_pmc_bytes_b128.md || exit $?
B=cuda-mpi-gpu-cluster-programming_amd/bin
for np in 2 4; do
  for ch in 1 0; do
    echo "== np $np chunks $ch" >> gpurun_out/r03_v5_halo.log
    timeout -k 10 240 $B/anxrun -np $np --timeout 200 $B/anx --version v5 --transport peer --batch 256 --iters 30 \
      --init rand --chunks $ch >> gpurun_out/r03_v5_halo.log 2>&1 || exit $?
  done
done
