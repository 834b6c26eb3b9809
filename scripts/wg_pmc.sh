# PMC (clock, MFMA busy) of the Winograd GEMM A/B arms: one counter pass with the kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=cuda-mpi-gpu-cluster-programming_amd/bin
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --kernel-trace --output-format csv -d gpurun_out/wgpmc -o run -- $B/anx_wgemm --images 300 --iters 3 \
  > gpurun_out/wgpmc.log 2>&1 && python3 tools/pmc_clock.py gpurun_out/wgpmc
