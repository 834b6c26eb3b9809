#!/bin/bash
# Cold-start probe (round 6): the bare HIP runtime's start-up (anx_hipinit, no libanx) under environment
# variants, the first-upload routes, and the anx --version v3 child. Outputs gpurun_out/r06/cold/.
B=cuda-mpi-gpu-cluster-programming_amd/bin
O=gpurun_out/r06/cold
mkdir -p $O
export TMPDIR=/tmp
j() { grep ANX_JSON | cut -c10-; }
{
for v in "" "GPU_MAX_HW_QUEUES=1" "GPU_MAX_HW_QUEUES=8" "HSA_ENABLE_SDMA=0" "ROCR_VISIBLE_DEVICES=0" "HIP_VISIBLE_DEVICES=0" "AMD_DIRECT_DISPATCH=0"; do
  for i in 1 2; do echo "env[$v] $(env $v timeout -k 5 60 $B/anx_hipinit | j)"; done
done
for m in pageable pinned kernel pageable pinned kernel; do echo "mode $m $(timeout -k 5 60 $B/anx_hipinit $m | j)"; done
for i in 1 2; do echo "anx v3 $(timeout -k 5 60 $B/anx --version v3 --batch 1 --init rand --iters 5 | j | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['cold_ms'], d.get('phases_cold'))")"; done
} > $O/cold2.log 2>&1
cat $O/cold2.log
