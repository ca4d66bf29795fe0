#!/bin/bash
# gpurun: TunableOp search for decode-batch projection GEMMs (M = decode batch), appended to the committed CSV.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp configs/tuning/tunableop_mi355x_gpt7b.csv gpurun_out/tun_dec.csv
for T in ${TOKENS:-1 8 16 32 64}; do
  timeout -k 10 300 python -u tools/gemm_tunable.py --tokens $T --ops fwd --skip-rocblas --append --csv gpurun_out/tun_dec.csv > gpurun_out/tune_dec_$T.log 2>&1 || { tail -20 gpurun_out/tune_dec_$T.log; exit 1; }
  grep "summary\|{\"hip" gpurun_out/tune_dec_$T.log | tail -1
done
