#!/bin/bash
# gpurun: attention tests, dK/dV ablation (unpipelined / pipelined / persistent) at B12 S2048,
# then the 1-GPU GPT-7B bench and a rocprofv3 kernel-stats profile of 3 steps.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q --timeout 120 --timeout-method thread -k "flash_attn or dkv or rope_flash or functional_autograd" > gpurun_out/attn_test.log 2>&1; rc=$?; tail -2 gpurun_out/attn_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_ablate.py 12 2048 32 128 > gpurun_out/ablate.log 2>&1 || { tail -5 gpurun_out/ablate.log; exit 1; }
grep "^{" gpurun_out/ablate.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_b1.log 2>&1 || { tail -20 gpurun_out/bench_b1.log; exit 1; }
tail -1 gpurun_out/bench_b1.log | cut -c1-300
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/prof_b1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_b1.log 2>&1 || { tail -20 gpurun_out/prof_b1.log; exit 1; }
  echo prof ok
fi
