#!/bin/bash
# gpurun: GPU tests, then bench.py A/B over env settings given as AB="NAME=VAL;NAME=VAL ..." (";"-separated runs)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
fi
IFS=';' read -ra RUNS <<< "${AB:-X=1}"
i=0
for run in "${RUNS[@]}"; do
  env $run timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err || { tail -20 gpurun_out/bench_$i.err; exit 1; }
  echo "[$run] $(cat gpurun_out/bench_$i.json)"
  i=$((i+1))
done
if [ -n "$PROF" ]; then
  R=$PWD
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
  echo prof ok
fi
