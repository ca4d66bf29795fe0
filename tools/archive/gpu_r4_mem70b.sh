#!/bin/bash
# gpurun: Llama-3-70B per-GPU memory of the PP4 x DP2 ZeRO-3 layout from 1-GPU slices vs the planner
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u tools/memory_check_70b.py --layers 1 2 --micro-batch 1 --ac selective > gpurun_out/mem70b.jsonl 2> gpurun_out/mem70b.err || { tail -30 gpurun_out/mem70b.err; exit 1; }
cat gpurun_out/mem70b.jsonl
