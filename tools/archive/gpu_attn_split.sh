#!/bin/bash
# gpurun: per-kernel attention backward split (ablation) at B12, then PMC passes of the kernels
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 200 python tools/attn_ablate.py 12 2048 32 128 > gpurun_out/attn_ablate.log 2>&1 || { tail -5 gpurun_out/attn_ablate.log; exit 1; }
tail -1 gpurun_out/attn_ablate.log
KINDS="${KINDS:-dkv dq fwd}" timeout -k 10 600 bash tools/gpu_attn_pmc2.sh | grep "fa_" | cut -c1-330
