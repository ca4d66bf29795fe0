#!/bin/bash
# gpurun: burst serving over scheduler policies / per-step token budgets, one process per arm
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for arm in ${ARMS:-prefill_first:4096 prefill_first:8192 prefill_first:16384 dynamic:8192 dynamic:16384}; do
  timeout -k 10 240 python -u tools/serve_budget_sweep.py $arm > gpurun_out/sweep_one.log 2>&1 || { tail -20 gpurun_out/sweep_one.log; exit 1; }
  grep '^{' gpurun_out/sweep_one.log | tee -a gpurun_out/serve_sweep.jsonl
done
