#!/bin/bash
# Round 6: prefill QKV GEMM with the RoPE / head-split epilogue (tail split through the reduce) -- tests + TTFT A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_fused_fwd.py tests/kernels/test_serving_gpu.py -k "qkv_rope or prefill or fused_forward or graph_decode" \
  > gpurun_out/r6_qkvrope_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ttft_ab.py --knob-sets prefill_qkv_rope=0 prefill_qkv_rope=1 --rounds 6 --repeats 4 \
  > gpurun_out/r6_qkvrope_ttft.log 2>&1
