#!/bin/bash
# gpurun: smoke, the whole GPU test suite, the driver-default bench, rocprofv3 kernel stats of the bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -20; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof_full
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_full.log 2>&1 || { tail -20 gpurun_out/prof_full.log; exit 1; }
echo prof ok
