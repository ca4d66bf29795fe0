#!/bin/bash
# gpurun: fused decode epilogue tests, then same-box A/B of the decode layer
# (LLMCTL_DECODE_FUSED=1 fused / =0 unfused): decode-step host breakdown + 16 x 2048 -> 128 burst
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py tests/kernels/test_serving_gpu.py -m gpu -x -q -k "fused or graph_decode" --timeout 120 --timeout-method thread > gpurun_out/fdec_tests.log 2>&1 || { tail -40 gpurun_out/fdec_tests.log; exit 1; }
tail -1 gpurun_out/fdec_tests.log
for run in 1 0 1 0; do
  LLMCTL_DECODE_FUSED=$run timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/fdec_host.json 2> gpurun_out/fdec_host.err || { tail -20 gpurun_out/fdec_host.err; exit 1; }
  echo "[fused=$run] $(cat gpurun_out/fdec_host.json)"
done
for run in 1 0; do
  LLMCTL_DECODE_FUSED=$run timeout -k 10 300 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=8192)
print(json.dumps(r), flush=True)
" > gpurun_out/fdec_ab.json 2> gpurun_out/fdec_ab.err || { tail -20 gpurun_out/fdec_ab.err; exit 1; }
  echo "[fused=$run] $(cut -c1-420 gpurun_out/fdec_ab.json)"
done
