#!/bin/bash
# gpurun: serving measurements (GPT-7B, 16 x 2048-token prompts): decode-step host breakdown,
# the 16 x 2048 -> 128 burst (llmctl bench e2e shape) + isolated TTFT, then rocprofv3 kernel
# stats of the decode-breakdown run (per decode step)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
R=$PWD
timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/serve_dec.json 2> gpurun_out/serve_dec.err || { tail -20 gpurun_out/serve_dec.err; exit 1; }
tail -1 gpurun_out/serve_dec.json
timeout -k 10 400 python -u -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark, single_request_ttft
r = run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                          scheduler='prefill_first', max_batch_tokens=4096)
print(json.dumps(r), flush=True)
print(json.dumps(single_request_ttft('gpt-7b', 2048)), flush=True)
" > gpurun_out/serve_e2e.jsonl 2> gpurun_out/serve_e2e.err || { tail -20 gpurun_out/serve_e2e.err; exit 1; }
cat gpurun_out/serve_e2e.jsonl
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/decprof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/decprof -o run -- python3 $R/tools/decode_host_breakdown.py > $R/gpurun_out/decprof.log 2>&1 || { tail -20 $R/gpurun_out/decprof.log; exit 1; }
  f=$(find $R/gpurun_out/decprof -name "*kernel_stats.csv" | head -1)
  python $R/tools/kstats.py "$f" 96 30 | tee $R/gpurun_out/decprof.txt
  cp "$f" $R/gpurun_out/decprof_kernel_stats.csv
  rm -rf $R/gpurun_out/decprof
fi
