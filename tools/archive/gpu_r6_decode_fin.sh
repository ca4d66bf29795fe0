#!/bin/bash
# Round 6: decode finalize inside the GEMM (knob decode_fin) -- tests, then an interleaved decode-step A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_kernels.py tests/kernels/test_serving_gpu.py \
  -k "decode_fin or fused or decode_qkv or up_swiglu or add_rmsnorm or add_sumsq or fp8_decode or graph_decode or async_decode_matches_sync" \
  > gpurun_out/r6_fin_tests.log 2>&1 || exit 1
for v in 0 1 0 1; do
  LLMCTL_KNOBS="decode_fin=$v" timeout -k 10 240 python -u tools/decode_host_breakdown.py --tokens 48 \
    > gpurun_out/r6_fin_ab_$v.$RANDOM.log 2>&1 || exit 1
done
LLMCTL_KNOBS="decode_fin=1" timeout -k 10 240 python -u tools/decode_host_breakdown.py --tokens 48 --weight-dtype fp8 --kv-cache-dtype fp8 \
  > gpurun_out/r6_fin_ab_fp8.log 2>&1
