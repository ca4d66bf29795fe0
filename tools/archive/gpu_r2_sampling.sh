#!/bin/bash
# gpurun: sampling + serving tests, then decode-step host breakdown and the CLI serving burst
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py tests/kernels/test_serving_gpu.py -m gpu -x -q -k "sampl or serving or graph or fused" --timeout 120 --timeout-method thread > gpurun_out/smp_tests.log 2>&1 || { tail -40 gpurun_out/smp_tests.log; exit 1; }
tail -1 gpurun_out/smp_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/smp_host.json 2> gpurun_out/smp_host.err || { tail -20 gpurun_out/smp_host.err; exit 1; }
  cat gpurun_out/smp_host.json
done
timeout -k 10 400 python -m llmctl bench e2e --prompt-length 2048 --gen-length 128 --num-requests 16 > gpurun_out/smp_e2e.json 2> gpurun_out/smp_e2e.err || { tail -20 gpurun_out/smp_e2e.err; exit 1; }
tr -d '\n ' < gpurun_out/smp_e2e.json | cut -c1-330; echo
