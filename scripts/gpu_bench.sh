#!/bin/bash
# Bench + profile session: headline bench (batch 128 and 256/GPU), full-AlexNet extension bench,
# kernel-trace profile, native CLI V3 cold/warm timings, conv micro-benchmarks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=cuda-mpi-gpu-cluster-programming_amd/bin
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch-per-gpu 256 > gpurun_out/bench1_b256.log 2>&1 && \
timeout -k 10 300 python bench.py --model full --steps 10 --warmup 3 --batch-per-gpu 256 > gpurun_out/bench_full.log 2>&1 && \
timeout -k 10 300 $B/anx --version v3 --iters 20 > gpurun_out/native_v3_b1.log 2>&1 && \
timeout -k 10 300 $B/anx --version v3 --batch 128 --init rand --iters 20 > gpurun_out/native_v3_b128.log 2>&1 && \
timeout -k 10 300 $B/anx_convbench --batch 64 --iters 20 > gpurun_out/convbench_direct.log 2>&1 && \
timeout -k 10 300 $B/anx_convbench --batch 64 --iters 20 --algo winograd --layer conv2 > gpurun_out/convbench_wino.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run -- python3 bench.py --model full --steps 5 --warmup 2 --batch-per-gpu 256 > gpurun_out/prof_full.log 2>&1
rc=$?
cat gpurun_out/smoke.log | tail -1; cat gpurun_out/bench1.log gpurun_out/bench1_b256.log gpurun_out/bench_full.log | grep metric
grep -h "ANX_JSON" gpurun_out/native_v3_*.log | cut -c1-300; grep -h "TFLOP" gpurun_out/convbench_*.log
exit $rc
