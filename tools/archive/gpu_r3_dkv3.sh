#!/bin/bash
# dK/dV A/B across sequence lengths after a kernel edit (+ the attention GPU tests first)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q --timeout 120 --timeout-method thread -k "flash_attn or dkv or rope_flash or functional_autograd" > gpurun_out/attn_test.log 2>&1; rc=$?; tail -2 gpurun_out/attn_test.log; [ $rc -eq 0 ] || exit $rc
for shp in "24 1024 32 128" "12 2048 32 128" "6 4096 32 128"; do
  timeout -k 10 120 python -u tools/attn_ablate.py $shp 2>&1 | grep "^{" || exit 1
done
