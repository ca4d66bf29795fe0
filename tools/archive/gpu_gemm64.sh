#!/bin/bash
# gpurun: gemm64_ex correctness + timing vs gemm_ex and hipBLASLt on the GPT-7B shapes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u tools/gemm64_bench.py ${ARGS} > gpurun_out/gemm64_bench.log 2>&1 || { tail -30 gpurun_out/gemm64_bench.log; exit 1; }
cat gpurun_out/gemm64_bench.log | grep -v '^{"tokens"'
