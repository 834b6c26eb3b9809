#!/bin/bash
# One build->measure iteration: all GPU tests, the 1-GPU benches (headline + bf16 extension), and
# kernel traces of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/it_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model full --batch-per-gpu 256 --steps 10 --warmup 3 > gpurun_out/it_bench_full.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/it_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/it_prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/it_prof_full -o run -- python3 bench.py --model full --batch-per-gpu 256 --steps 5 --warmup 2 > gpurun_out/it_prof_full.log 2>&1
rc=$?
tail -3 gpurun_out/it_pytest.log; tail -1 gpurun_out/it_bench.log; tail -1 gpurun_out/it_bench_full.log
python3 tools/rocprof_summary.py gpurun_out/it_prof/run_results.db --steps 13 2>/dev/null | head -8
python3 tools/rocprof_summary.py gpurun_out/it_prof_full/run_results.db --steps 7 2>/dev/null | head -14
exit $rc
