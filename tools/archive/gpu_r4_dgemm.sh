#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/decode_gemm_bw.py ${ARGS} > gpurun_out/dgemm.jsonl 2> gpurun_out/dgemm.err || { tail -20 gpurun_out/dgemm.err; exit 1; }
cat gpurun_out/dgemm.jsonl
