#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q --timeout 120 --timeout-method thread -k "norm or rms or layer" > gpurun_out/norm_tests.log 2>&1 || { tail -30 gpurun_out/norm_tests.log; exit 1; }
tail -1 gpurun_out/norm_tests.log
timeout -k 10 300 python -u tools/elementwise_bench.py > gpurun_out/elementwise.log 2>&1 || { tail -20 gpurun_out/elementwise.log; exit 1; }
cat gpurun_out/elementwise.log
