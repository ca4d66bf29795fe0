#!/bin/bash
# gpurun: fused-forward GEMM epilogue tests, then a same-box GPT-7B step A/B (LLMCTL_FUSED_FWD 0 / 1).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_fused_fwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_fused_test.log 2>&1 || { tail -40 gpurun_out/r3_fused_test.log; exit 1; }
tail -2 gpurun_out/r3_fused_test.log
for v in ${AB:-0 1 0 1}; do
  LLMCTL_FUSED_FWD=$v timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_fused$v.log 2>&1 || { tail -20 gpurun_out/bench_fused$v.log; exit 1; }
  echo "FUSED_FWD=$v $(tail -1 gpurun_out/bench_fused$v.log | cut -c1-200)"
done
