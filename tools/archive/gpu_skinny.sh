#!/bin/bash
# gpurun: kernel GPU tests, decode kernel bench (paged attention + decode GEMMs), serving e2e A/B
# (weight-streaming decode GEMM on / off).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/kernels -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_kernels.log 2>&1 || { tail -40 gpurun_out/gpu_tests_kernels.log; exit 1; }
tail -2 gpurun_out/gpu_tests_kernels.log
timeout -k 10 300 python -u tools/decode_bench.py --json-out gpurun_out/decode_bench.jsonl > gpurun_out/decode_bench.log 2>&1 || { tail -20 gpurun_out/decode_bench.log; exit 1; }
grep gemm gpurun_out/decode_bench.jsonl
for sk in ${SKS:-1 0}; do
LLMCTL_SKINNY_GEMM=$sk timeout -k 10 400 python -u -c "
import json, sys
sys.path.insert(0, '.')
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16)), flush=True)
" > gpurun_out/serve_bench_sk$sk.json 2> gpurun_out/serve_bench_sk$sk.err || { tail -20 gpurun_out/serve_bench_sk$sk.err; exit 1; }
echo "skinny=$sk $(cat gpurun_out/serve_bench_sk$sk.json)"
done
