#!/bin/bash
# gpurun: kernel-time profiles of the serving paths: single 2048-token prefill (TTFT) and the
# 16 x 2048 -> 128 burst (prefill + graph-replayed decode).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ttft -o ttft -- \
  python3 tools/ttft_bench.py --repeats 5 > gpurun_out/prof_ttft.log 2>&1 || { tail -20 gpurun_out/prof_ttft.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e -o e2e -- \
  python3 -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=2048)))
" > gpurun_out/prof_e2e.log 2>&1 || { tail -20 gpurun_out/prof_e2e.log; exit 1; }
find gpurun_out/prof_ttft gpurun_out/prof_e2e -name "*kernel_stats.csv" | head
