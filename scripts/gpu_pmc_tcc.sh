#!/bin/bash
# L2 (TCC) counters of the 1-GPU bench step: hit/miss in one pass, FETCH_SIZE (3 TCC counters) in another.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/tcc1 -o pmc -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/tcc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tcc2 -o pmc -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/tcc2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/tcc3 -o pmc -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/tcc3.log 2>&1
rc=$?
ls -R gpurun_out/tcc* | head
exit $rc
