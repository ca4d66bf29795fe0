#!/bin/bash
# One-wave-per-SIMD GEMM (gemm_w4) vs gemm64 vs hipBLASLt on the GPT-7B projection shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gemm64_bench.py --no-old --groups 4 --rounds 5 --w4 ${W4CFG:-4 204} > gpurun_out/w4_bench.log 2>&1
rc=$?
tail -n 8 gpurun_out/w4_bench.log
exit $rc
