#!/bin/bash
# gpurun: same-box bench A/B (gemm64 tail split on / off), then attention PMC passes + attn bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for run in "LLMCTL_GEMM64_CONFIG=104" "LLMCTL_GEMM64_CONFIG=1104" "LLMCTL_GEMM64_CONFIG=104"; do
  env $run timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "[$run] $(cut -c1-200 gpurun_out/ab.json)"
done
for args in "--B 8" "--B 12"; do
  timeout -k 10 120 python -u tools/attn_bench.py $args 2>&1 | tail -1
done
KINDS="fwd dkv dq" timeout -k 10 600 bash tools/gpu_attn_pmc.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmcattn > gpurun_out/pmcattn_summary.txt 2>&1
cat gpurun_out/pmcattn_summary.txt
