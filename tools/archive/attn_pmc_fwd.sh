# PMC counters of the flash-attention forward at B16 S2048 H32 D128 causal: the default kernel
# (fa_w64 = 0) and the asm one-wave-per-SIMD kernel (fa_w64 = 3); one counter set per pass.
set -o pipefail
R=$PWD
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmcfwd
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  for w in 0 3; do
    i=$((i+1))
    ATTN_KNOBS=fa_w64=$w timeout -k 10 -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcfwd/w$w.$i -o run --output-format csv -- python3 $R/tools/attn_one.py fwd 5 16 2048 32 128 > $R/gpurun_out/pmcfwd/w$w.$i.log 2>&1 || { echo "fail w$w $set"; tail -5 $R/gpurun_out/pmcfwd/w$w.$i.log; exit 1; }
  done
done
echo done
