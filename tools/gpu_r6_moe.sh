#!/bin/bash
# Round 6: MoE expert rows padded to multiples of 256 (gemm64 expert GEMMs) and linear() routing every
# gradient-needing projection through _Linear -- GPU tests, then the Mixtral-8x7B slice A/B (moe_pad 1 / 0).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/kernels/test_kernels.py tests/kernels/test_fused_fwd.py -k "moe or linear or fused or gemm64" \
  > gpurun_out/r6_moe_tests.log 2>&1 || exit 1
: > gpurun_out/r6_moe_slice.log
for p in 1 0 1 0; do
  LLMCTL_KNOBS=moe_pad=$p timeout -k 10 300 python tools/slice_bench.py --model mixtral-8x7b --layers 1 3 --micro-batch 4 \
    --steps 4 --warmup 2 2>&1 | grep '^{' | sed "s/^{/{\"moe_pad\": $p, /" >> gpurun_out/r6_moe_slice.log || exit 1
done
