#!/bin/bash
# gpurun: rocprofv3 kernel stats of the GPT-7B step for each knob set in $ARMS (';'-separated
# LLMCTL_KNOBS strings; empty = defaults), 3 profiled steps (+2 warm-up) each
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
export TMPDIR=/tmp
IFS=';' read -ra arms <<< "$ARMS"
n=0
for k in "${arms[@]}"; do
  n=$((n+1))
  rm -rf gpurun_out/prof_arm$n
  LLMCTL_KNOBS="$k" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_arm$n -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_arm$n.log 2>&1 || { tail -20 gpurun_out/prof_arm$n.log; exit 1; }
  f=$(find gpurun_out/prof_arm$n -name "*kernel_stats.csv" | head -1)
  echo "== arm $n [$k]: $(tail -1 gpurun_out/prof_arm$n.log | cut -c1-150)"
  grep '"metric"' gpurun_out/prof_arm$n.log | cut -c1-200
  python tools/kstats.py "$f" 5 ${TOP:-25} | tee gpurun_out/prof_arm$n.txt
  cp "$f" gpurun_out/prof_arm${n}_kernel_stats.csv
  rm -rf gpurun_out/prof_arm$n
done
