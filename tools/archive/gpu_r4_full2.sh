#!/bin/bash
# gpurun: smoke, whole GPU suite, default bench, then a 2-round A/B of the wgrad GEMM kernel
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
bash tools/gpu_r4_full.sh || exit 1
A_KNOBS="gemm64_config=104" B_KNOBS="gemm64_config=804" ROUNDS=2 bash tools/gpu_r4_ab.sh
