#!/bin/bash
# gpurun: Llama-3-70B decoder-layer slice (real dims) fwd+bwd+AdamW, then the serving e2e burst
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u tools/slice_bench.py --model llama-70b --layers 2 6 --micro-batch 2 > gpurun_out/slice70b_r3.jsonl 2> gpurun_out/slice70b_r3.err || { tail -20 gpurun_out/slice70b_r3.err; exit 1; }
cat gpurun_out/slice70b_r3.jsonl
timeout -k 10 400 python -u -c "
import json, os
from llmctl.benchmarks.serving import run_serving_benchmark, single_request_ttft
r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                          scheduler='prefill_first', max_batch_tokens=4096)
print(json.dumps(r), flush=True)
print(json.dumps(single_request_ttft('gpt-7b', 2048)), flush=True)
" > gpurun_out/serve_e2e_r3b.jsonl 2> gpurun_out/serve_e2e_r3b.err || { tail -20 gpurun_out/serve_e2e_r3b.err; exit 1; }
cat gpurun_out/serve_e2e_r3b.jsonl
