#!/bin/bash
# gpurun: gemm64 tests, the 1-GPU GPT-7B bench, then a rocprofv3 kernel-stats profile of 3 steps.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm64.py tests/kernels/test_fused_fwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_gemm_test.log 2>&1 || { tail -30 gpurun_out/r3_gemm_test.log; exit 1; }
tail -1 gpurun_out/r3_gemm_test.log
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_r3.log 2>&1 || { tail -20 gpurun_out/bench_r3.log; exit 1; }
tail -1 gpurun_out/bench_r3.log | cut -c1-300
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/prof_r3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_r3.log 2>&1 || { tail -20 gpurun_out/prof_r3.log; exit 1; }
  find gpurun_out/prof_r3 -name "*kernel_stats.csv" | head -3
fi
