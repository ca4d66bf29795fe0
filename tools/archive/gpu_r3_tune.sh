#!/bin/bash
# gpurun: TunableOp search for the GPT-7B forward + W^T data-gradient (TN) GEMMs at 32768 tokens
# (micro-batch 16) and the W^T data gradients at 24576 tokens (micro-batch 12)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 700 python -u tools/gemm_tunable.py --tokens 32768 --ops fwd,dgradT --skip-rocblas --csv gpurun_out/tun_32k.csv --json gpurun_out/tun_32k.json > gpurun_out/tun_32k.log 2>&1 || { tail -20 gpurun_out/tun_32k.log; exit 1; }
grep -E "tunableop|hipblaslt|summary" gpurun_out/tun_32k.log | tail -25
timeout -k 10 500 python -u tools/gemm_tunable.py --tokens 24576 --ops dgradT --skip-rocblas --csv gpurun_out/tun_24k.csv --json gpurun_out/tun_24k.json > gpurun_out/tun_24k.log 2>&1 || { tail -20 gpurun_out/tun_24k.log; exit 1; }
grep -E "tunableop|hipblaslt" gpurun_out/tun_24k.log | tail -12
