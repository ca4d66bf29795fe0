#!/bin/bash
# gpurun: attention kernel numerics, then backward/forward timings.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -v --timeout 120 --timeout-method thread -k "flash or packed" > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
timeout -k 10 200 python -u tools/attn_ablate.py > gpurun_out/attn_ablate.log 2>&1 || { tail -20 gpurun_out/attn_ablate.log; exit 1; }
cat gpurun_out/attn_ablate.log
