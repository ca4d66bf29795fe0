#!/bin/bash
# Round 6: kernel breakdown of the Mixtral-8x7B layer-slice training step (rocprofv3 --kernel-trace --stats).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_moe -o run -- \
  python3 $R/tools/slice_bench.py --model mixtral-8x7b --layers 1 2 --micro-batch 4 --steps 4 --warmup 2 \
  > $R/gpurun_out/prof_moe.log 2>&1
