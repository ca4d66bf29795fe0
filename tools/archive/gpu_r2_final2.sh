#!/bin/bash
# gpurun (round 2 close): smoke, all GPU tests, 1-GPU bench (driver defaults), bench kernel stats,
# serving burst through the CLI defaults (llmctl bench e2e: prefill_first, 4096-token budget)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 python -m llmctl bench e2e --prompt-length 2048 --gen-length 128 --num-requests 16 > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
tr -d '\n ' < gpurun_out/e2e.json | cut -c1-500; echo
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
echo prof ok
