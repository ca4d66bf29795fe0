#!/bin/bash
# Round 6: burst serving (16 x 2048 -> 128, prefill_first, 4096-token budget) with / without the folded
# prefill RMSNorm, interleaved, one process per arm.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
: > gpurun_out/r6_nf_burst.log
for nf in 0 1 0 1; do
  LLMCTL_KNOBS=prefill_norm_fold=$nf timeout -k 10 300 python -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark(model='gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                          scheduler='prefill_first')
r['arm'] = 'prefill_norm_fold=$nf'
print(json.dumps(r))
" 2>&1 | grep '^{' >> gpurun_out/r6_nf_burst.log || exit 1
done
