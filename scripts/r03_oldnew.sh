# In-box A/B of the round-2 library (abl/libanx_r02.so) against the current one, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
one() {  # one NAME LIB ARGS...
  local name=$1 lib=$2; shift 2
  if [ "$lib" = old ]; then export ANX_LIB=$PWD/abl/libanx_r02.so ANX_WINO_SPLIT=0; else unset ANX_LIB ANX_WINO_SPLIT; fi
  timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-b1 "$@" > gpurun_out/on_$name.log 2>&1 || exit 1
  python3 -c "import json; r=json.loads(open('gpurun_out/on_$name.log').read().strip().splitlines()[-1]); print('$name', '$*', r['value'], r['ms_per_step'])"
}
for i in 1 2 3; do one old$i old; one new$i new; done
for i in 1 2; do one old64_$i old --batch-per-gpu 64; one new64_$i new --batch-per-gpu 64 --lanes 2; done
