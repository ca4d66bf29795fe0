#!/bin/bash
# gpurun: after retiring the losing gemm64 variants -- gemm tests + shape bench of the survivors,
# then smoke + the whole GPU suite + the driver-default bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/kernels/test_gemm64.py tests/kernels/test_fused_fwd.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/retire_test.log 2>&1 || { tail -40 gpurun_out/retire_test.log; exit 1; }
tail -1 gpurun_out/retire_test.log
timeout -k 10 300 python -u tools/gemm4w_bench.py --configs 104 304 904 > gpurun_out/retire_bench.log 2>&1 || { tail -20 gpurun_out/retire_bench.log; exit 1; }
grep '^{' gpurun_out/retire_bench.log
bash tools/gpu_r4_full.sh
