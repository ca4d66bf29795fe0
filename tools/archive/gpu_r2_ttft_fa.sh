#!/bin/bash
# gpurun: serving GPU tests, then single-request TTFT (2k prompt) A/B of the prefill attention
# (LLMCTL_PREFILL_FA=1: flash attention, one prompt -> plain causal with K/V split; =0 paged kernel)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_serving_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tf_tests.log 2>&1 || { tail -30 gpurun_out/tf_tests.log; exit 1; }
tail -1 gpurun_out/tf_tests.log
for run in 1 0 1 0; do
  echo "[fa=$run] $(LLMCTL_PREFILL_FA=$run timeout -k 10 200 python -u tools/ttft_bench.py 2>/dev/null | tail -1)"
done
