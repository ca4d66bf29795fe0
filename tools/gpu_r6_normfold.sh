#!/bin/bash
# Round 6: serving prefill with the RMSNorm folded into the QKV / gate-up GEMMs (row-scaled epilogue) --
# kernel + engine tests, the existing gemm64 / fused / serving tests, then a single-prompt TTFT A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_norm_fold.py tests/kernels/test_fused_fwd.py tests/kernels/test_gemm64.py \
  > gpurun_out/r6_nf_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_serving_gpu.py -k "prefill or graph_decode or fused" \
  > gpurun_out/r6_nf_serving.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ttft_ab.py --init-knobs prefill_norm_fold=1 \
  --knob-sets prefill_norm_fold=0 prefill_norm_fold=1 --rounds 6 --repeats 4 \
  > gpurun_out/r6_nf_ttft.log 2>&1
