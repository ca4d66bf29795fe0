#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/kernels/test_kernels.py -x -q -k "flash or functional" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.json 2> gpurun_out/attn_bench.err || { tail -20 gpurun_out/attn_bench.err; exit 1; }
cat gpurun_out/attn_bench.json
