#!/bin/bash
# gpurun: gemm64 SwiGLU-epilogue + serving tests, then same-box A/B (LLMCTL_PREFILL_SWIGLU=1/0) of
# the single 2k-prompt TTFT and the 16 x 2048 burst (CLI defaults)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py tests/kernels/test_serving_gpu.py tests/kernels/test_gemm64.py -m gpu -x -q -k "swiglu or serving or graph or prefill or gemm64" --timeout 120 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || { tail -40 gpurun_out/ps_tests.log; exit 1; }
tail -1 gpurun_out/ps_tests.log
for run in 1 0 1 0; do
  echo "[swiglu=$run] $(LLMCTL_PREFILL_SWIGLU=$run timeout -k 10 200 python -u tools/ttft_bench.py 2>/dev/null | tail -1)"
done
for run in 1 0; do
  LLMCTL_PREFILL_SWIGLU=$run timeout -k 10 400 python -m llmctl bench e2e --prompt-length 2048 --gen-length 128 --num-requests 16 > gpurun_out/ps_e2e.json 2> gpurun_out/ps_e2e.err || { tail -20 gpurun_out/ps_e2e.err; exit 1; }
  echo "[swiglu=$run] $(tr -d '\n ' < gpurun_out/ps_e2e.json | cut -c1-330)"
done
