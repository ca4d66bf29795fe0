#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -u tools/gemm_tunable.py --tokens 24576 --csv gpurun_out/tunableop_gpt7b.csv --json gpurun_out/gemm_tunable.json > gpurun_out/gemm_tunable.log 2>&1; rc=$?; tail -60 gpurun_out/gemm_tunable.log; exit $rc
