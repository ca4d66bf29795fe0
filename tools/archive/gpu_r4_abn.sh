#!/bin/bash
# gpurun: interleaved GPT-7B bench over N knob sets ($ARMS: ';'-separated LLMCTL_KNOBS strings,
# an empty one = defaults), ROUNDS rounds (default 2)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
IFS=';' read -ra arms <<< "$ARMS"
for i in $(seq 1 ${ROUNDS:-2}); do
  for k in "${arms[@]}"; do
    LLMCTL_KNOBS="$k" timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "[$k] $(tail -1 gpurun_out/ab.log | cut -c1-170)" | tee -a gpurun_out/abn.log
  done
done
