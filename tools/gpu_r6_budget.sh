#!/bin/bash
# Round 6: burst serving (16 x 2048 -> 128, prefill_first) per-step token budget 4096 vs 6144, interleaved, one process per arm.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_budget.log
for b in 4096 6144 4096 6144; do
  timeout -k 10 300 python -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark(model='gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                          scheduler='prefill_first', max_batch_tokens=$b)
r['arm'] = 'prefill_first:$b'
print(json.dumps(r))
" 2>&1 | grep '^{' >> gpurun_out/r6_budget.log || exit 1
done
