#!/bin/bash
# pool2+LRN wave kernels (fp32 headline, bf16 full model) with a capped, looping grid vs one wave per
# pixel: LRN/engine/full-model tests, then interleaved bench A/B over the grid cap.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_full_alexnet.py tests/test_gpu_engine.py -k "lrn or full or engine or golden" > gpurun_out/lc_tests.log 2>&1 || { tail -30 gpurun_out/lc_tests.log; exit 1; }
tail -2 gpurun_out/lc_tests.log
for r in 1 2; do
  for c in 0 2048 1024 4096; do
    ANX_LRN_WAVE_WGS=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/lc_b_${c}_$r.log 2>&1 || exit $?
    ANX_LRN_WAVE_WGS=$c timeout -k 10 300 python bench.py --model full --steps 30 --warmup 5 > gpurun_out/lc_f_${c}_$r.log 2>&1 || exit $?
    echo "cap $c round $r: blocks $(grep '"metric"' gpurun_out/lc_b_${c}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])') full $(grep '"metric"' gpurun_out/lc_f_${c}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lc_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/lc_prof.log 2>&1
