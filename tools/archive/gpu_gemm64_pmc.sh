#!/bin/bash
# PMC counters for gemm64 vs hipBLASLt (counters only; no trace domains). One pass per set.
set -o pipefail
mkdir -p gpurun_out/pmc64
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" ; do
  for kind in ${KINDS:-fwd dgrad torch_fwd}; do
    i=$((i+1))
    timeout -k 10 -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmc64/$kind.$i -o run --output-format csv -- python3 $R/tools/gemm64_one.py $kind ${CFG:-104} 20 > $R/gpurun_out/pmc64/$kind.$i.log 2>&1 || { echo "fail $kind $set"; tail -5 $R/gpurun_out/pmc64/$kind.$i.log; exit 1; }
  done
done
echo done
