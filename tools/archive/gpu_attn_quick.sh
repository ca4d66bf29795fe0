#!/bin/bash
# gpurun: attention kernel tests + fwd/bwd throughput (B12 S2048 H32 D128 causal; B1 S2048 prefill)
# for each env setting in ENVS (";"-separated), then for every abtmp/*.so build (same-box A/B)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
IFS=';' read -ra RUNS <<< "${ENVS:-X=1}"
for run in "${RUNS[@]}"; do
  echo "=== $run"
  env $run timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -m gpu -x -q -k "flash or attn or packed" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
  tail -1 gpurun_out/attn_tests.log
  for args in "--B 12" "--B 12" "--B 1 --iters 50"; do
    env $run timeout -k 10 120 python -u tools/attn_bench.py $args 2>&1 | tail -1 | cut -c1-200
  done
done
for so in abtmp/*.so; do
  echo "--- $so"
  for args in "--B 12" "--B 1 --iters 50"; do
    LLMCTL_HIP_LIB=$PWD/$so timeout -k 10 120 python -u tools/attn_bench.py $args 2>&1 | tail -1 | cut -c1-200
  done
done
