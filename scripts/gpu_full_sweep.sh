#!/bin/bash
# Full AlexNet bf16 extension: images per GPU sweep and a kernel trace at the default batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 256 512 1024; do
  timeout -k 10 300 python bench.py --model full --steps 20 --warmup 5 --batch-per-gpu $b > gpurun_out/fs_$b.log 2>&1 || exit $?
  echo "B $b: $(grep '"metric"' gpurun_out/fs_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["tflops"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/full_prof -o run -- python3 bench.py --model full --steps 10 --warmup 3 --batch-per-gpu 256 > gpurun_out/full_prof.log 2>&1
