#!/bin/bash
# gpurun: attention tests on the current library, then attn_ablate timing of the current vs a
# previous build ($ALT, LLMCTL_HIP_LIB), interleaved
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q --timeout 120 --timeout-method thread -k "flash_attn or dkv or rope_flash or functional_autograd" > gpurun_out/aab_test.log 2>&1; rc=$?; tail -1 gpurun_out/aab_test.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in "" "$ALT"; do
    LLMCTL_HIP_LIB=$lib timeout -k 10 120 python -u tools/attn_ablate.py ${ABL_B:-16} 2048 32 128 > gpurun_out/aab.log 2>&1 || { tail -5 gpurun_out/aab.log; exit 1; }
    echo "[${lib:-current}] $(grep '^{' gpurun_out/aab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["flash_attn_fwd_op"]["ms"], "dq", d["dq"]["ms"], "dkv", d["dkv"]["ms"], "bwd_op", d["flash_attn_bwd_op"]["ms"])')"
  done
done
