#!/bin/bash
# gpurun: serving GPU tests (TP=2 / TP=8 processes on one GPU, fused decode) + custom all-reduce tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests/kernels/test_serving_gpu.py tests/kernels/test_custom_ar_gpu.py -x -v --timeout 400 --timeout-method thread ${K:+-k "$K"} > gpurun_out/r3_serve_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r3_serve_test.log | tail -40; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r3_serve_test.log | tail -40; tail -2 gpurun_out/r3_serve_test.log
