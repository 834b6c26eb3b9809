#!/bin/bash
# A/B: bench.py default (2 lanes x 300, eager) vs the same step captured in a HIP graph, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 --graph $g > gpurun_out/gl_${g}_$r.log 2>&1 || exit $?
    echo "graph $g round $r: $(grep '"metric"' gpurun_out/gl_${g}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["hip_graph"])')"
  done
done
