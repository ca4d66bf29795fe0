#!/bin/bash
# gpurun: attention/RoPE kernel tests + fused RoPE-attention backward, then bench A/B fused vs unfused
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -m gpu -x -q -k "flash or attn or rope or packed" --timeout 120 --timeout-method thread > gpurun_out/ra_tests.log 2>&1 || { tail -30 gpurun_out/ra_tests.log; exit 1; }
tail -1 gpurun_out/ra_tests.log
for run in "LLMCTL_FUSED_ROPE_ATTN=1" "LLMCTL_FUSED_ROPE_ATTN=0" "LLMCTL_FUSED_ROPE_ATTN=1" "LLMCTL_FUSED_ROPE_ATTN=0"; do
  env $run timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "[$run] $(cut -c1-150 gpurun_out/ab.json)"
done
