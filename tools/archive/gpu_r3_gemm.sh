#!/bin/bash
# gpurun: gemm64 correctness (every variant) then the leading-dimension / schedule-variant probe.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_gemm64.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_gemm_test.log 2>&1 || { tail -30 gpurun_out/r3_gemm_test.log; exit 1; }
tail -3 gpurun_out/r3_gemm_test.log
timeout -k 10 500 python -u tools/gemm_ld_probe.py ${ARGS:---configs 104 404} > gpurun_out/ld_probe.log 2>&1 || { tail -30 gpurun_out/ld_probe.log; exit 1; }
cat gpurun_out/ld_probe.log
