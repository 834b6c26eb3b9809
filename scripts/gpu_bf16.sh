#!/bin/bash
# bf16 full-AlexNet: LDS-DMA ring kernel tests, then the extension bench per kernel mode (ANX_BF16_GLDS)
# and a kernel trace of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_full_alexnet.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/bf16_pytest.log 2>&1 && \
ANX_BF16_GLDS=0 timeout -k 10 300 python bench.py --model full --batch-per-gpu 256 --steps 10 --warmup 3 > gpurun_out/bf16_bench0.log 2>&1 && \
ANX_BF16_GLDS=2 timeout -k 10 300 python bench.py --model full --batch-per-gpu 256 --steps 10 --warmup 3 > gpurun_out/bf16_bench2.log 2>&1 && \
ANX_BF16_GLDS=3 timeout -k 10 300 python bench.py --model full --batch-per-gpu 256 --steps 10 --warmup 3 > gpurun_out/bf16_bench3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bf16_prof -o run -- python3 bench.py --model full --batch-per-gpu 256 --steps 5 --warmup 2 > gpurun_out/bf16_prof.log 2>&1
rc=$?
tail -3 gpurun_out/bf16_pytest.log
for m in 0 2 3; do echo "mode $m: $(tail -1 gpurun_out/bf16_bench$m.log | cut -c1-220)"; done
exit $rc
