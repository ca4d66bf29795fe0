#!/bin/bash
# gpurun: rocprofv3 kernel stats of a decode-heavy serving run
# (NREQ x PLEN-token prompts, GEN new tokens; defaults 16 x 2048 -> 256).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
cat > /tmp/decode_run.py <<PY
import sys, json
sys.path.insert(0, "$R")
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=${PLEN:-2048}, gen_length=${GEN:-256}, num_requests=${NREQ:-16}, max_batch_size=${NREQ:-16})), flush=True)
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_decode -o run --output-format csv -- python3 /tmp/decode_run.py > $R/gpurun_out/prof_decode.log 2>&1 || { tail -20 $R/gpurun_out/prof_decode.log; exit 1; }
tail -1 $R/gpurun_out/prof_decode.log
