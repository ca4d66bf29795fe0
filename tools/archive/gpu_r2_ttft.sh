#!/bin/bash
# gpurun: serving TTFT A/B (gemm64 small-M forward on / off) + burst benchmark over prefill budgets
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_serving_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/serve_tests.log 2>&1 || { tail -30 gpurun_out/serve_tests.log; exit 1; }
tail -1 gpurun_out/serve_tests.log
for run in "LLMCTL_FWD64=1" "LLMCTL_FWD64=0"; do
  echo "[$run] $(env $run timeout -k 10 200 python -u tools/ttft_bench.py 2>/dev/null | tail -1)"
done
timeout -k 10 800 python -u -c "
import json, sys
from llmctl.benchmarks.serving import run_serving_benchmark
for mbt in (2048, 4096, 8192):
    r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=mbt)
    print(json.dumps(r), flush=True)
" > gpurun_out/serve_bench_r2b.jsonl 2> gpurun_out/serve_bench.err || { tail -20 gpurun_out/serve_bench.err; exit 1; }
cut -c1-330 gpurun_out/serve_bench_r2b.jsonl
