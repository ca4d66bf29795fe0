#!/bin/bash
# gpurun: gemm_ex numerics, then gemm_ex vs hipBLASLt on the GPT-7B shapes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/kernels/test_kernels.py -x -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -3 gpurun_out/gemm_tests.log
timeout -k 10 400 python tools/gemm_bench.py ${ROUNDS:-5} > gpurun_out/gemm_bench.json 2> gpurun_out/gemm_bench.err || { tail -20 gpurun_out/gemm_bench.err; exit 1; }
cat gpurun_out/gemm_bench.json
