#!/bin/bash
# gpurun: bench A/B of the data-gradient path: gemm64 dgrad (W read K-major, fused SwiGLU
# epilogue) vs W^T copy + hipBLASLt forward-layout GEMM (LLMCTL_DGRAD64=0)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for run in "LLMCTL_DGRAD64=1" "LLMCTL_DGRAD64=0" "LLMCTL_DGRAD64=1" "LLMCTL_DGRAD64=0"; do
  env $run timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "[$run] $(cut -c1-150 gpurun_out/ab.json)"
done
