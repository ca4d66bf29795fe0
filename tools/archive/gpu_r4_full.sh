#!/bin/bash
# gpurun: smoke, the whole GPU test suite (driver form, verbose), the driver-default bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -20; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
