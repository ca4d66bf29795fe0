#!/bin/bash
# gpurun: serving e2e on GPT-7B (16 x 2048 -> 128 burst, prefill_first / 4096-token budget, mixed
# steps on and off) + isolated-request TTFT; then the TP=8 eight-process serving test alone.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u -c "
import json, os
from llmctl.benchmarks.serving import run_serving_benchmark, single_request_ttft
for mixed in ('1', '0', '1'):
    os.environ['LLMCTL_MIXED_STEPS'] = mixed
    r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                              scheduler='prefill_first', max_batch_tokens=4096)
    r['mixed_steps_env'] = mixed
    print(json.dumps(r), flush=True)
os.environ['LLMCTL_MIXED_STEPS'] = '1'
print(json.dumps(single_request_ttft('gpt-7b', 2048)), flush=True)
" > gpurun_out/serve_e2e_r3.jsonl 2> gpurun_out/serve_e2e_r3.err || { tail -20 gpurun_out/serve_e2e_r3.err; exit 1; }
cat gpurun_out/serve_e2e_r3.jsonl
if [ -n "$TP8" ]; then
  LLMCTL_HANG_DUMP=200 timeout -k 10 450 python -u -m pytest tests/kernels/test_serving_gpu.py -x -v --timeout 420 --timeout-method thread -k tp8 > gpurun_out/tp8_test.log 2>&1; rc=$?
  grep -E "PASSED|FAILED|passed|failed" gpurun_out/tp8_test.log | tail -5
  exit $rc
fi
