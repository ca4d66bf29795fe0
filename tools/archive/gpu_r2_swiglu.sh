#!/bin/bash
# gpurun: gemm64 + fused-SwiGLU tests, then bench A/B fused vs unfused SwiGLU backward
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm64.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g64_tests.log 2>&1 || { tail -30 gpurun_out/g64_tests.log; exit 1; }
tail -1 gpurun_out/g64_tests.log
for run in "LLMCTL_FUSED_SWIGLU=1" "LLMCTL_FUSED_SWIGLU=0" "LLMCTL_FUSED_SWIGLU=1" "LLMCTL_FUSED_SWIGLU=0"; do
  env $run timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "[$run] $(cut -c1-150 gpurun_out/ab.json)"
done
