#!/bin/bash
# gpurun: 4-wave GEMM correctness (gemm64 tests incl. variant 6) + shape bench, then the full suite + bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm64.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g4w_test.log 2>&1 || { tail -30 gpurun_out/g4w_test.log; exit 1; }
tail -2 gpurun_out/g4w_test.log
timeout -k 10 300 python -u tools/gemm4w_bench.py --configs 104 404 804 904 > gpurun_out/g4w_bench.log 2>&1 || { tail -20 gpurun_out/g4w_bench.log; exit 1; }
cat gpurun_out/g4w_bench.log
bash tools/gpu_r4_full.sh
