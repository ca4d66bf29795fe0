#!/bin/bash
# Round 6: tail split for the serving gate/up + SwiGLU GEMM -- tests, then a burst A/B (native knob
# swiglu_fwd_split 1 / 0, interleaved processes) and a single-prompt TTFT check.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_norm_fold.py tests/kernels/test_kernels.py -k "swiglu or rowscale or rstd or norm_fold or linear_acc" \
  > gpurun_out/r6_sw_tests.log 2>&1 || exit 1
: > gpurun_out/r6_sw_burst.log
for sw in 1 0 1 0; do
  timeout -k 10 300 python -c "
import json, torch
from llmctl.ops import _lib
assert _lib.load()
torch.ops.llmctl.set_knob('swiglu_fwd_split', $sw)
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark(model='gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                          scheduler='prefill_first')
r['arm'] = 'swiglu_fwd_split=$sw'
print(json.dumps(r))
" 2>&1 | grep '^{' >> gpurun_out/r6_sw_burst.log || exit 1
done
