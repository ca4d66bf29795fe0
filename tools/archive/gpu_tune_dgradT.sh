#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp configs/tuning/tunableop_mi355x_gpt7b.csv gpurun_out/tun3.csv
timeout -k 10 700 python -u tools/gemm_tunable.py --tokens 24576 --ops dgrad,dgradT --skip-rocblas --append --csv gpurun_out/tun3.csv > gpurun_out/tune_dgradT.log 2>&1; rc=$?; grep -v "^tuned\|amdgpu" gpurun_out/tune_dgradT.log | tail -30; exit $rc
