#!/bin/bash
# One gpurun call: kernel tests, attention bench, short 7B bench, rocprof stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/kernels -x -q > gpurun_out/kernel_tests.log 2>&1; echo "kernel tests rc=$?" >> gpurun_out/kernel_tests.log
tail -5 gpurun_out/kernel_tests.log
