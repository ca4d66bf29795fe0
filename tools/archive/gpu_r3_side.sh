#!/bin/bash
# gpurun: side-job SwiGLU backward — kernel tests, standalone timing, then GPT-7B step A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm64.py -x -q --timeout 120 --timeout-method thread -k "swiglu" > gpurun_out/side_test.log 2>&1; rc=$?; tail -3 gpurun_out/side_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/swiglu_side_bench.py > gpurun_out/side_bench.log 2>&1 || { tail -20 gpurun_out/side_bench.log; exit 1; }
cat gpurun_out/side_bench.log | grep "^{"
if [ -n "$AB" ]; then
for m in side epilogue side epilogue; do
  LLMCTL_SWIGLU_BWD=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/bench_$m.log | cut -c1-200)"
done
fi
