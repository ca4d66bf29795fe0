#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/kernels/test_kernels.py -x -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 400 python tools/gemm_variants.py ${ROUNDS:-5} $VARIANTS > gpurun_out/gemm_variants.json 2> gpurun_out/gemm_variants.err || { tail -20 gpurun_out/gemm_variants.err; exit 1; }
head -3 gpurun_out/gemm_variants.json
