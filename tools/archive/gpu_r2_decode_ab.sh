#!/bin/bash
# gpurun: decode GEMM kernel tests, then serving burst A/B of the decode GEMM routing
# (LLMCTL_SKINNY_GEMM=1: LDS-staged v2 for every projection at 5-16 tokens; =narrow: previous)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -m gpu -x -q -k "decode_gemm or skinny" --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
for run in "LLMCTL_SKINNY_GEMM=1" "LLMCTL_SKINNY_GEMM=narrow" "LLMCTL_SKINNY_GEMM=1" "LLMCTL_SKINNY_GEMM=narrow"; do
  env $run timeout -k 10 300 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=8192)
print(json.dumps(r), flush=True)
" > gpurun_out/dec_ab.json 2> gpurun_out/dec_ab.err || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "[$run] $(cut -c1-400 gpurun_out/dec_ab.json)"
done
