# bench.py A/B: interleaved runs over LLMCTL_KNOBS settings given as AB="knobs;knobs;..." (";"-separated runs;
# "-" = defaults), each bench under its own time limit; results in gpurun_out/ab_*.json
set -o pipefail
mkdir -p gpurun_out
IFS=';' read -ra RUNS <<< "${AB:--}"
i=0
for run in "${RUNS[@]}"; do
  k="$run"; [ "$k" = "-" ] && k=""
  LLMCTL_KNOBS="$k" timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 8 --warmup 3} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -20 gpurun_out/ab_$i.err; exit 1; }
  echo "[$run] $(cut -c1-200 gpurun_out/ab_$i.json)"
  i=$((i+1))
done
