#!/bin/bash
# gpurun: register-staged-B 4-wave GEMM (variant 5): gemm tests, shape bench vs 904 / hipBLASLt
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest tests/kernels/test_gemm64.py tests/kernels/test_fused_fwd.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/il4_test.log 2>&1 || { tail -40 gpurun_out/il4_test.log; exit 1; }
tail -2 gpurun_out/il4_test.log
timeout -k 10 300 python -u tools/gemm4w_bench.py --configs 904 504  # 504 = retired register-staged variant; see profiles/gemm_regstage_ab_r4.txt > gpurun_out/il4_bench.log 2>&1 || { tail -20 gpurun_out/il4_bench.log; exit 1; }
grep '^{' gpurun_out/il4_bench.log
