set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=cuda-mpi-gpu-cluster-programming_amd/bin
timeout -k 10 120 $B/anx_wgemm --images 300 --iters 20 > gpurun_out/wg300.log 2>&1 && \
timeout -k 10 120 $B/anx_wgemm --images 64 --iters 20 > gpurun_out/wg64.log 2>&1
rc=$?
cat gpurun_out/wg300.log gpurun_out/wg64.log
exit $rc
