#!/bin/bash
# gpurun: gemm64 tests, full GPU suite, then the 7B bench with gemm64 on vs off (A/B).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm64.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm64_tests.log 2>&1 || { tail -40 gpurun_out/gemm64_tests.log; exit 1; }
tail -1 gpurun_out/gemm64_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for g in 1 0 1; do
  LLMCTL_GEMM64=$g timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_g64_$g.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  echo "gemm64=$g $(cat gpurun_out/bench_g64_$g.json)"
done
