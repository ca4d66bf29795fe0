#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u tools/mem_breakdown.py --model llama3-70b --layers 1 2 > gpurun_out/membd.jsonl 2> gpurun_out/membd.err || { tail -30 gpurun_out/membd.err; exit 1; }
cat gpurun_out/membd.jsonl
