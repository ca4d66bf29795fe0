set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q --timeout 120 --timeout-method thread -k "flash_attn or dkv or rope_flash or functional_autograd" > gpurun_out/attn_test.log 2>&1; rc=$?; tail -3 gpurun_out/attn_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/attn_ablate.py 12 2048 32 128 > gpurun_out/attn_ablate.log 2>&1; rc=$?; cat gpurun_out/attn_ablate.log | grep -v amdgpu.ids; exit $rc
