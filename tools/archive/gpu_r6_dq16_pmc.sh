# round 6: PMC of the dQ kernel, 32x32x16 (dq16=0) vs 16x16x32 (dq16=1)
set -o pipefail
mkdir -p gpurun_out/pmcdq16
R=$PWD
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  export ATTN_KNOBS=dq16=$m
  timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcdq16/dq.$m -o run --output-format csv -- python3 $R/tools/attn_one.py dq 20 16 2048 32 128 > $R/gpurun_out/pmcdq16/dq.$m.log 2>&1 || { echo "fail $m"; tail -5 $R/gpurun_out/pmcdq16/dq.$m.log; exit 1; }
done
cd $R && python tools/pmc_summary.py gpurun_out/pmcdq16 fa_bwd_dq > gpurun_out/pmcdq16_summary.txt 2>&1; cat gpurun_out/pmcdq16_summary.txt
