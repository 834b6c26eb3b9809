set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in 2 3 4 1; do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --lanes $L --no-b1 > gpurun_out/lanes_$L.log 2>&1 || exit 1
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/lanes_$L.log').read().strip().splitlines()[-1]); print('lanes', $L, r['value'], r['ms_per_step'])"
done
timeout -k 10 120 python bench.py --steps 50 --warmup 5 --lanes 2 --batch-per-gpu 256 --no-b1 > gpurun_out/lanes_2_256.log 2>&1 && tail -1 gpurun_out/lanes_2_256.log | cut -c1-200
