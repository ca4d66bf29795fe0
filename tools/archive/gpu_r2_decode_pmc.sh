#!/bin/bash
# gpurun: rocprofv3 passes over the decode GEMM (fused-path v3 kernel) on uncached GPT-7B weights:
# kernel stats, then HBM bytes (FETCH_SIZE) + active cycles
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dgpmc_t -o run --output-format csv -- python3 $R/tools/decode_gemm_pmc.py 20 > $R/gpurun_out/dgpmc_t.log 2>&1 || { tail -20 $R/gpurun_out/dgpmc_t.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/dgpmc_c -o run --output-format csv -- python3 $R/tools/decode_gemm_pmc.py 20 > $R/gpurun_out/dgpmc_c.log 2>&1 || { tail -20 $R/gpurun_out/dgpmc_c.log; exit 1; }
echo ok
