#!/bin/bash
# gpurun: GEMM / training / stream-check GPU tests, then same-box bench A/B of the side-stream
# W^T refresh (LLMCTL_WT_SIDE_STREAM=1/0)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "gemm64 or linear or stream or train or engine or multirank or zero or tp" --timeout 120 --timeout-method thread > gpurun_out/wt_tests.log 2>&1 || { tail -40 gpurun_out/wt_tests.log; exit 1; }
tail -1 gpurun_out/wt_tests.log
for run in 1 0 1 0; do
  LLMCTL_WT_SIDE_STREAM=$run timeout -k 10 400 python bench.py > gpurun_out/wt.json 2> gpurun_out/wt.err || { tail -20 gpurun_out/wt.err; exit 1; }
  echo "[wt_side=$run] $(sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*"max_mem_gb": ([0-9.]+).*/\1 tok\/s \2 ms \3 GB/' gpurun_out/wt.json)"
done
