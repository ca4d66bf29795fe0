#!/bin/bash
# dK/dV kernel study: per-FLOP rate vs sequence length (fixed-cost share) + PMC of the pipelined
# and unpipelined kernels at B12 S2048.
set -o pipefail
mkdir -p gpurun_out/pmcdkv
export PYTHONPATH=$PWD
R=$PWD
for shp in "24 1024 32 128" "12 2048 32 128" "6 4096 32 128"; do
  timeout -k 10 120 python -u tools/attn_ablate.py $shp 2>&1 | grep "^{" || exit 1
done
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
  for kind in dkv_old dkv_pipe; do
    i=$((i+1))
    timeout -k 10 -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcdkv/$kind.$i -o run --output-format csv -- python3 $R/tools/attn_one.py $kind 5 12 2048 32 128 > $R/gpurun_out/pmcdkv/$kind.$i.log 2>&1 || { echo "fail $kind"; tail -5 $R/gpurun_out/pmcdkv/$kind.$i.log; exit 1; }
  done
done
cd $R && python tools/pmc_summary.py gpurun_out/pmcdkv fa_bwd > gpurun_out/pmcdkv_summary.txt 2>&1; cat gpurun_out/pmcdkv_summary.txt
