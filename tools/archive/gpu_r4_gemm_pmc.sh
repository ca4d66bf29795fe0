#!/bin/bash
# PMC counters of the GEMM kernels (one pass per counter set): hipBLASLt vs gemm64 configs on one
# GPT-7B shape / layout -> gpurun_out/gemmpmc_summary.txt
set -o pipefail
mkdir -p gpurun_out/gemmpmc
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  for c in ${CFGS:-torch 104 904}; do
    i=$((i+1))
    timeout -k 10 -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/gemmpmc/$c.$i -o run --output-format csv -- python3 $R/tools/gemm64_one.py ${KIND:-fwd} $c 10 ${SHAPE:-up} > $R/gpurun_out/gemmpmc/$c.$i.log 2>&1 || { echo "fail $c $set"; tail -5 $R/gpurun_out/gemmpmc/$c.$i.log; exit 1; }
  done
done
cd $R && python tools/pmc_summary.py gpurun_out/gemmpmc "${KSUB:-}" > gpurun_out/gemmpmc_summary.txt 2>&1; cat gpurun_out/gemmpmc_summary.txt
