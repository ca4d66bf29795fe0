# round 6: GEMM tests (incl. the in-kernel split-K reduction) + prefill TTFT A/B (fused split on / off)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/kernels/test_gemm64.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_gemm_tests.log 2>&1 &&
tail -2 gpurun_out/r6_gemm_tests.log &&
timeout -k 10 400 python -u tools/gemm4w_bench.py --tokens 2048 --configs 304 --layouts fwd --knob-sets gemm_fused_split=0 > gpurun_out/r6_split_bench.log 2>&1 &&
grep '^{' gpurun_out/r6_split_bench.log &&
timeout -k 10 300 python -u tools/ttft_ab.py --knob-sets gemm_fused_split=0 gemm_fused_split=1 > gpurun_out/r6_ttft_ab.log 2>&1 &&
grep '^{' gpurun_out/r6_ttft_ab.log
