#!/bin/bash
# gpurun: decode-step time vs paged-attention context splits (16 x 2k, fused decode layer)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for sp in 1 2 3 0 2 1 0; do
  if [ "$sp" = "0" ]; then unset LLMCTL_DECODE_SPLITS; else export LLMCTL_DECODE_SPLITS=$sp; fi
  timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/sw_host.json 2> gpurun_out/sw_host.err || { tail -20 gpurun_out/sw_host.err; exit 1; }
  echo "[splits=${sp:-auto}] $(cat gpurun_out/sw_host.json)"
done
