#!/bin/bash
# gpurun: serving e2e benchmarks (decode-heavy and prefill-heavy) on GPT-7B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
for kw in [dict(prompt_length=128, gen_length=256, num_requests=64, max_batch_size=64),
           dict(prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16)]:
    print(json.dumps(run_serving_benchmark('gpt-7b', **kw)), flush=True)
" > gpurun_out/serve_bench.jsonl 2> gpurun_out/serve_bench.err || { tail -20 gpurun_out/serve_bench.err; exit 1; }
cat gpurun_out/serve_bench.jsonl
