#!/bin/bash
# Round 6: MoE expert data gradients on gemm64 (unsinked weights, no W^T copy) vs hipBLASLt NN (knob dgrad64=off):
# MoE GPU tests, then the Mixtral-8x7B slice A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/kernels/test_kernels.py tests/kernels/test_fused_fwd.py -k "moe or linear or fused" \
  > gpurun_out/r6_moe2_tests.log 2>&1 || exit 1
: > gpurun_out/r6_moe2_slice.log
for k in "dgrad64=fused" "dgrad64=off" "dgrad64=fused" "dgrad64=off"; do
  LLMCTL_KNOBS=$k timeout -k 10 300 python tools/slice_bench.py --model mixtral-8x7b --layers 1 3 --micro-batch 4 \
    --steps 4 --warmup 2 2>&1 | grep '^{' | sed "s/^{/{\"knobs\": \"$k\", /" >> gpurun_out/r6_moe2_slice.log || exit 1
done
