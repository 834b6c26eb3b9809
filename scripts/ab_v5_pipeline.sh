set -e
B=cuda-mpi-gpu-cluster-programming_amd/bin
O=gpurun_out/v5ab; mkdir -p $O
for rep in 1 2; do
for np in 2 4; do
for split in rows hybrid; do
for pipe in on off; do
  timeout -k 10 120 $B/anxrun -np $np --timeout 100 $B/anx --version v5 --transport peer --split $split --batch 64 --iters 30 --pipeline $pipe --init rand > $O/run.log 2>&1
  echo "np=$np split=$split pipe=$pipe $(grep ANX_JSON $O/run.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[9:]); print(r["warm_ms"], {k: round(v,3) for k,v in r["phases_warm"].items()})')" | tee -a $O/ab.txt
done; done; done; done
