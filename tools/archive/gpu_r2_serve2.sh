#!/bin/bash
# gpurun: serving GPU tests (incl. TP=2 two-process custom-AR graph test) + serving bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/kernels/test_serving_gpu.py tests/kernels/test_kernels.py -x -v --timeout 200 --timeout-method thread > gpurun_out/serve_gpu_tests.log 2>&1 || { tail -40 gpurun_out/serve_gpu_tests.log; exit 1; }
tail -1 gpurun_out/serve_gpu_tests.log
timeout -k 10 600 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
for kw in [dict(scheduler='prefill_first', max_batch_tokens=8192), dict(scheduler='prefill_first', max_batch_tokens=2048)]:
    r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, **kw)
    print(json.dumps(r), flush=True)
r = run_serving_benchmark('gpt-7b', prompt_length=128, gen_length=256, num_requests=1, max_batch_size=1)
print(json.dumps(r), flush=True)
" > gpurun_out/serve_bench_r2b.jsonl 2> gpurun_out/serve_bench.err || { tail -20 gpurun_out/serve_bench.err; exit 1; }
cat gpurun_out/serve_bench_r2b.jsonl
