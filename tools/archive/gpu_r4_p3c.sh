#!/bin/bash
# gpurun: persistent GEMM (peeled tail, drain knob): race hunt, gemm tests, bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/debug_p3b.py 16 > gpurun_out/dbg.log 2>&1 || { tail -20 gpurun_out/dbg.log; exit 1; }
cat gpurun_out/dbg.log
timeout -k 10 500 python -u -m pytest tests/kernels/test_gemm64.py tests/kernels/test_fused_fwd.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/p3_test.log 2>&1 || { tail -40 gpurun_out/p3_test.log; exit 1; }
tail -2 gpurun_out/p3_test.log
timeout -k 10 300 python -u tools/gemm4w_bench.py --configs 904 304 > gpurun_out/p3_bench.log 2>&1 || { tail -20 gpurun_out/p3_bench.log; exit 1; }
cat gpurun_out/p3_bench.log
timeout -k 10 300 python -u tools/gemm4w_bench.py --configs 304 --knob gemm_p3_drain=0 > gpurun_out/p3_bench_nd.log 2>&1 || { tail -20 gpurun_out/p3_bench_nd.log; exit 1; }
cat gpurun_out/p3_bench_nd.log
