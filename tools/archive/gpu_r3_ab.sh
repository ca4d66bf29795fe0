#!/bin/bash
# gpurun: attention + gemm64 tests, then an interleaved GPT-7B bench A/B of env setting $A_ENV vs $B_ENV
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q --timeout 120 --timeout-method thread -k "flash_attn or dkv or rope_flash or functional_autograd" > gpurun_out/ab_test.log 2>&1; rc=$?; tail -1 gpurun_out/ab_test.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for e in "$A_ENV" "$B_ENV"; do
    env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "[$e] $(tail -1 gpurun_out/ab.log | cut -c1-170)"
  done
done
