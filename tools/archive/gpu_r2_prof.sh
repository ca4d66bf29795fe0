#!/bin/bash
# gpurun: rocprofv3 kernel stats of the 1-GPU GPT-7B bench (3 timed steps) -> per-step summary
mkdir -p gpurun_out
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
grep metric $R/gpurun_out/prof_bench.log | cut -c1-200
