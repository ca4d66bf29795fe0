#!/bin/bash
# gpurun: TunableOp search for the serving prefill projection shapes, appended to the committed CSV.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp configs/tuning/tunableop_mi355x_gpt7b.csv gpurun_out/tun.csv
for T in ${TOKENS:-2048}; do
  timeout -k 10 500 python -u tools/gemm_tunable.py --tokens $T --ops fwd --skip-rocblas --append --csv gpurun_out/tun.csv --json gpurun_out/tune_$T.json > gpurun_out/tune_$T.log 2>&1 || { tail -20 gpurun_out/tune_$T.log; exit 1; }
  grep -v "^tuned" gpurun_out/tune_$T.log | tail -12
done
