#!/bin/bash
# gpurun: kernel stats of the 16 x 2048 -> 128 serving burst (decode steps are graph replays)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/decprof -o run --output-format csv -- python3 -c "
import json, sys
sys.path.insert(0, '$R')
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=8192)))
" > $R/gpurun_out/decprof.log 2>&1 || { tail -20 $R/gpurun_out/decprof.log; exit 1; }
grep tpot $R/gpurun_out/decprof.log | cut -c1-400
