#!/bin/bash
# gpurun: attention forward knob A/B (workgroup shape) and the bench at micro-batch 16 vs 12
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for e in LLMCTL_FA_NW=4 LLMCTL_FA_NW=8 LLMCTL_FA_NW=4 LLMCTL_FA_NW=8; do
  env $e timeout -k 10 120 python -u tools/attn_ablate.py 12 2048 32 128 > gpurun_out/kn.log 2>&1 || { tail -5 gpurun_out/kn.log; exit 1; }
  echo "[$e] $(grep '^{' gpurun_out/kn.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["flash_attn_fwd_op"], d["dq"], d["dkv"])')"
done
for mb in 16 12; do
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --micro-batch $mb > gpurun_out/kb.log 2>&1 || { tail -5 gpurun_out/kb.log; exit 1; }
  echo "[mb $mb] $(tail -1 gpurun_out/kb.log | cut -c1-150) $(tail -1 gpurun_out/kb.log | grep -o '"max_mem_gb": [0-9.]*')"
done
