# round 6: dQ on MFMA 16x16x32 -- numerics (fp32 oracle, vs the 32x32x16 kernel) then timing A/B
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/kernels/test_kernels.py -x -q -k "dq16 or flash_attn" --timeout 200 --timeout-method thread > gpurun_out/r6_dq16_tests.log 2>&1 &&
tail -2 gpurun_out/r6_dq16_tests.log &&
timeout -k 10 300 python -u tools/dq16_ab.py > gpurun_out/r6_dq16_ab.log 2>&1 &&
grep '^{' gpurun_out/r6_dq16_ab.log
