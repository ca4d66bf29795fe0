#!/bin/bash
# gpurun: attention kernel tests + fwd/bwd throughput (B8 S2048 H32 D128 causal; B1 S2048 prefill)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -m gpu -x -q -k "flash or attn" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for args in "--B 8" "--B 8" "--B 1 --iters 50"; do
  timeout -k 10 120 python -u tools/attn_bench.py $args 2>&1 | tail -1
done
if [ -f abtmp/base.so ]; then
  echo "--- baseline build"
  for args in "--B 8" "--B 8" "--B 1 --iters 50"; do
    LLMCTL_HIP_LIB=$PWD/abtmp/base.so timeout -k 10 120 python -u tools/attn_bench.py $args 2>&1 | tail -1
  done
fi
