#!/bin/bash
# PMC counters for the gemm kernels (counters only; no trace domains).
set -o pipefail
mkdir -p gpurun_out/pmc
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" ; do
  for kind in wgrad fwd torch_wgrad torch_fwd; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set -d $R/gpurun_out/pmc/$kind.$i -o run --output-format csv -- python3 $R/tools/gemm_one.py $kind -1 3 > $R/gpurun_out/pmc/$kind.$i.log 2>&1 || { echo "fail $kind $set"; tail -5 $R/gpurun_out/pmc/$kind.$i.log; exit 1; }
  done
done
echo done
