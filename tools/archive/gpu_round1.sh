#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/kernels -q -rf > gpurun_out/kernel_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc" | tee -a gpurun_out/kernel_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 180 python tools/attn_bench.py --iters 5 > gpurun_out/attn_bench.json 2> gpurun_out/attn_bench.err || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 2 --micro-batch 4 > gpurun_out/bench_mb4.json 2> gpurun_out/bench_mb4.err || exit $?
