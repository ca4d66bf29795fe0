#!/bin/bash
# gpurun: effective shader clock per kernel during the 7B training step (GRBM_GUI_ACTIVE cycles / kernel time).
set -o pipefail
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc_clock -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/pmc_clock.log 2>&1 || { tail -20 $R/gpurun_out/pmc_clock.log; exit 1; }
ls $R/gpurun_out/pmc_clock
