#!/bin/bash
# gpurun: GPU tests, bench (mb sweep), rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for mb in ${MBS:-8}; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --micro-batch $mb > gpurun_out/bench_mb$mb.json 2> gpurun_out/bench_mb$mb.err || { tail -20 gpurun_out/bench_mb$mb.err; exit 1; }
  cat gpurun_out/bench_mb$mb.json
done
if [ -n "$PROF" ]; then
  R=$PWD
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --micro-batch ${PMB:-8} > $R/gpurun_out/prof_bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
  echo prof ok
fi
