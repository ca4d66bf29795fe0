#!/bin/bash
# gpurun: same-box A/B of training-step knobs on the 1-GPU GPT-7B bench (driver config)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for run in "LLMCTL_DGRAD64=fused" "X=1" "LLMCTL_DGRAD64=0" "LLMCTL_DGRAD64=fused" "X=1" "LLMCTL_DGRAD64=0"; do
  env $run timeout -k 10 400 python bench.py > gpurun_out/knob.json 2> gpurun_out/knob.err || { tail -20 gpurun_out/knob.err; exit 1; }
  echo "[$run] $(cut -c1-200 gpurun_out/knob.json)"
done
