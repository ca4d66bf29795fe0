#!/bin/bash
# Round 6: per-kernel prefill tables (rocprofv3 --kernel-trace --stats) with and without the folded RMSNorm.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
export LLMCTL_KNOBS=prefill_norm_fold=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nf0 -o run -- \
  python3 $R/tools/ttft_bench.py --repeats 5 > $R/gpurun_out/prof_nf0.log 2>&1 || exit 1
export LLMCTL_KNOBS=prefill_norm_fold=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nf1 -o run -- \
  python3 $R/tools/ttft_bench.py --repeats 5 > $R/gpurun_out/prof_nf1.log 2>&1
