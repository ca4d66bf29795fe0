#!/bin/bash
# gpurun: fused-QKV decode attention tests, then same-box A/B (LLMCTL_DECODE_ATTN_QKV=1/0) of the
# decode step (host breakdown) and the serving burst (CLI defaults)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py tests/kernels/test_serving_gpu.py -m gpu -x -q -k "fused or graph_decode or paged or decode" --timeout 120 --timeout-method thread > gpurun_out/aq_tests.log 2>&1 || { tail -40 gpurun_out/aq_tests.log; exit 1; }
tail -1 gpurun_out/aq_tests.log
for run in 1 0 1 0; do
  LLMCTL_DECODE_ATTN_QKV=$run timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/aq_host.json 2> gpurun_out/aq_host.err || { tail -20 gpurun_out/aq_host.err; exit 1; }
  echo "[attn_qkv=$run] $(cat gpurun_out/aq_host.json)"
done
for run in 1 0; do
  LLMCTL_DECODE_ATTN_QKV=$run timeout -k 10 400 python -m llmctl bench e2e --prompt-length 2048 --gen-length 128 --num-requests 16 > gpurun_out/aq_e2e.json 2> gpurun_out/aq_e2e.err || { tail -20 gpurun_out/aq_e2e.err; exit 1; }
  echo "[attn_qkv=$run] $(tr -d '\n ' < gpurun_out/aq_e2e.json | cut -c1-330)"
done
