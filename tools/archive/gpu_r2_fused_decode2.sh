#!/bin/bash
# gpurun: decode GEMM + fused epilogue tests, then same-box A/B: fused layer on the v3 GEMM
# (weight loads before x staging) vs v2, and unfused; decode-step GPU time (host breakdown) + burst
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py tests/kernels/test_serving_gpu.py -m gpu -x -q -k "fused or graph_decode or decode_gemm or skinny" --timeout 120 --timeout-method thread > gpurun_out/fdec_tests.log 2>&1 || { tail -40 gpurun_out/fdec_tests.log; exit 1; }
tail -1 gpurun_out/fdec_tests.log
for run in "LLMCTL_DECODE_FUSED=1 LLMCTL_DECODE_V3=1" "LLMCTL_DECODE_FUSED=1 LLMCTL_DECODE_V3=0" "LLMCTL_DECODE_FUSED=0 LLMCTL_DECODE_V3=0" "LLMCTL_DECODE_FUSED=1 LLMCTL_DECODE_V3=1" "LLMCTL_DECODE_FUSED=1 LLMCTL_DECODE_V3=0" "LLMCTL_DECODE_FUSED=0 LLMCTL_DECODE_V3=0"; do
  env $run timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/fdec_host.json 2> gpurun_out/fdec_host.err || { tail -20 gpurun_out/fdec_host.err; exit 1; }
  echo "[$run] $(cat gpurun_out/fdec_host.json)"
done
for run in "LLMCTL_DECODE_FUSED=1 LLMCTL_DECODE_V3=1" "LLMCTL_DECODE_FUSED=0 LLMCTL_DECODE_V3=0"; do
  env $run timeout -k 10 300 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=8192)
print(json.dumps(r), flush=True)
" > gpurun_out/fdec_ab.json 2> gpurun_out/fdec_ab.err || { tail -20 gpurun_out/fdec_ab.err; exit 1; }
  echo "[$run] $(cut -c1-420 gpurun_out/fdec_ab.json)"
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fdecprof3 -o run --output-format csv -- python3 $R/tools/decode_host_breakdown.py > $R/gpurun_out/fdecprof3.log 2>&1 || { tail -20 $R/gpurun_out/fdecprof3.log; exit 1; }
echo prof ok
