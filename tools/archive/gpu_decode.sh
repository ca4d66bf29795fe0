#!/bin/bash
# gpurun: kernel + serving GPU tests, paged-decode bandwidth sweep, serving e2e bench
# (16 x 2048-token prompts, 128 new tokens), copy-site profile of a 4-layer training step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/kernels -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_kernels.log 2>&1 || { tail -40 gpurun_out/gpu_tests_kernels.log; exit 1; }
tail -2 gpurun_out/gpu_tests_kernels.log
timeout -k 10 300 python -u tools/decode_bench.py --json-out gpurun_out/decode_bench.jsonl > gpurun_out/decode_bench.log 2>&1 || { tail -20 gpurun_out/decode_bench.log; exit 1; }
cat gpurun_out/decode_bench.jsonl
timeout -k 10 300 python -u tools/decode_bench.py --hkv 4 --hq 4 --json-out gpurun_out/decode_bench_tp8.jsonl > gpurun_out/decode_bench_tp8.log 2>&1 || { tail -20 gpurun_out/decode_bench_tp8.log; exit 1; }
cat gpurun_out/decode_bench_tp8.jsonl
timeout -k 10 400 python -u -c "
import json, sys
sys.path.insert(0, '.')
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16)), flush=True)
" > gpurun_out/serve_bench.json 2> gpurun_out/serve_bench.err || { tail -20 gpurun_out/serve_bench.err; exit 1; }
cat gpurun_out/serve_bench.json
if [ -n "$AB1" ]; then
  LLMCTL_DECODE_SPLITS=1 timeout -k 10 400 python -u -c "
import json, sys
sys.path.insert(0, '.')
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16)), flush=True)
" > gpurun_out/serve_bench_split1.json 2> gpurun_out/serve_bench_split1.err || { tail -20 gpurun_out/serve_bench_split1.err; exit 1; }
  cat gpurun_out/serve_bench_split1.json
fi
if [ -n "$COPIES" ]; then
  timeout -k 10 300 python -u tools/find_copies.py > gpurun_out/find_copies.log 2>&1 || { tail -20 gpurun_out/find_copies.log; exit 1; }
  head -40 gpurun_out/find_copies.log
fi
