#!/bin/bash
# gpurun: serving GPU tests, then same-box TTFT A/B of fresh-prompt prefill attention
# (LLMCTL_PREFILL_FA=1 packed flash attention / =0 paged-prefill kernel)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_serving_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pfa_tests.log 2>&1 || { tail -40 gpurun_out/pfa_tests.log; exit 1; }
tail -1 gpurun_out/pfa_tests.log
for run in 1 0 1 0; do
  LLMCTL_PREFILL_FA=$run timeout -k 10 300 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=8192)
print(json.dumps(r), flush=True)
" > gpurun_out/pfa_ab.json 2> gpurun_out/pfa_ab.err || { tail -20 gpurun_out/pfa_ab.err; exit 1; }
  echo "[fa=$run] $(cut -c1-330 gpurun_out/pfa_ab.json)"
done
