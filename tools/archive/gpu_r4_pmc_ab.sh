#!/bin/bash
# gpurun: GEMM PMC (hipBLASLt vs gemm64 104 / 904, up-projection forward + wgrad), then the step A/B of
# the weight-gradient kernel (gemm64_config 104 vs 904)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
CFGS="torch 104 904" KIND=fwd SHAPE=up bash tools/gpu_r4_gemm_pmc.sh > gpurun_out/gemmpmc_fwd.txt 2>&1 || { tail -20 gpurun_out/gemmpmc_fwd.txt; exit 1; }
cp gpurun_out/gemmpmc_summary.txt gpurun_out/gemmpmc_summary_fwd.txt
rm -rf gpurun_out/gemmpmc
CFGS="torch 104 904" KIND=wgrad SHAPE=up bash tools/gpu_r4_gemm_pmc.sh > gpurun_out/gemmpmc_wgrad.txt 2>&1 || { tail -20 gpurun_out/gemmpmc_wgrad.txt; exit 1; }
cp gpurun_out/gemmpmc_summary.txt gpurun_out/gemmpmc_summary_wgrad.txt
rm -rf gpurun_out/gemmpmc
A_KNOBS="gemm64_config=104" B_KNOBS="gemm64_config=904" ROUNDS=2 bash tools/gpu_r4_ab.sh
