#!/bin/bash
# gpurun: serving burst (16 x 2048-token prompts -> 128 tokens) under the scheduling policies.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
i=0
for cfg in "dynamic 8192" "prefill_first 8192" "prefill_first 2048"; do
  set -- $cfg
  timeout -k 10 400 python -u -c "
import json, sys
sys.path.insert(0, '.')
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='$1', max_batch_tokens=$2)), flush=True)
" > gpurun_out/serve_policy_$i.json 2> gpurun_out/serve_policy_$i.err || { tail -20 gpurun_out/serve_policy_$i.err; exit 1; }
  cat gpurun_out/serve_policy_$i.json
  i=$((i+1))
done
