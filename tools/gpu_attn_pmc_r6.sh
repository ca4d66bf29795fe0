#!/bin/bash
# PMC counters of the flash-attention kernels (counters only; one pass per set) -> summary.
set -o pipefail
mkdir -p gpurun_out/pmcattn6
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  for kind in ${KINDS:-fwd dkv dq}; do
    i=$((i+1))
    timeout -k 10 -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcattn6/$kind.$i -o run --output-format csv -- python3 $R/tools/attn_one.py $kind 5 ${ABL_B:-16} 2048 32 128 > $R/gpurun_out/pmcattn6/$kind.$i.log 2>&1 || { echo "fail $kind $set"; tail -5 $R/gpurun_out/pmcattn6/$kind.$i.log; exit 1; }
  done
done
cd $R && python tools/pmc_summary.py gpurun_out/pmcattn6 fa_ > gpurun_out/pmcattn6_summary.txt 2>&1; cat gpurun_out/pmcattn6_summary.txt
