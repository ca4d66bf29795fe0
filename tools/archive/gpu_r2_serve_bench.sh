#!/bin/bash
# gpurun: serving e2e benchmark on GPT-7B (16 x 2048 -> 128 burst; both schedulers; budgets) +
# isolated-request TTFT.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -c "
import json, sys
from llmctl.benchmarks.serving import run_serving_benchmark, single_request_ttft
for kw in [dict(scheduler='prefill_first', max_batch_tokens=8192), dict(scheduler='dynamic', max_batch_tokens=8192),
           dict(scheduler='prefill_first', max_batch_tokens=16384)]:
    r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, **kw)
    print(json.dumps(r), flush=True)
print(json.dumps(single_request_ttft('gpt-7b', 2048)), flush=True)
" > gpurun_out/serve_bench_r2.jsonl 2> gpurun_out/serve_bench.err || { tail -20 gpurun_out/serve_bench.err; exit 1; }
cat gpurun_out/serve_bench_r2.jsonl
