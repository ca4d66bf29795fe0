#!/bin/bash
# gpurun: burst serving (prefill_first:4096) under prefill GEMM routing knob sets ($KSETS: ';'-separated
# LLMCTL_KNOBS strings, empty = defaults), one process per arm, two rounds
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
IFS=';' read -ra ks <<< "${KSETS:-;prefill_swiglu=0;fwd64=all;fwd64=off}"
for i in 1 2; do
  for k in "${ks[@]}"; do
    LLMCTL_KNOBS="$k" timeout -k 10 240 python -u tools/serve_budget_sweep.py prefill_first:4096 > gpurun_out/sk_one.log 2>&1 || { tail -20 gpurun_out/sk_one.log; exit 1; }
    echo "[$k] $(grep '^{' gpurun_out/sk_one.log)" | tee -a gpurun_out/serve_knobs.log
  done
done
