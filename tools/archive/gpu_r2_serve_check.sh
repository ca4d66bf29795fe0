#!/bin/bash
# gpurun: all GPU tests, then decode-step host breakdown + serving burst (fused decode, incremental
# prefix indexing, cached sampling parameters)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/sc_host.json 2> gpurun_out/sc_host.err || { tail -20 gpurun_out/sc_host.err; exit 1; }
  cat gpurun_out/sc_host.json
done
timeout -k 10 300 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
for kw in (dict(num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=8192), dict(num_requests=16, max_batch_size=16, scheduler='dynamic', max_batch_tokens=8192)):
    r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, **kw)
    print(json.dumps(r), flush=True)
" > gpurun_out/sc_burst.jsonl 2> gpurun_out/sc_burst.err || { tail -20 gpurun_out/sc_burst.err; exit 1; }
cut -c1-420 gpurun_out/sc_burst.jsonl
