#!/bin/bash
# gpurun: serving GPU tests (paged prefill kernel, chunked prefill, prefix cache), then smoke.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/kernels/test_serving_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/serve_gpu_tests.log 2>&1 || { tail -40 gpurun_out/serve_gpu_tests.log; exit 1; }
tail -1 gpurun_out/serve_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
