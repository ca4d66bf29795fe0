set -o pipefail
timeout -k 10 400 python -u tools/gemm4w_bench.py --configs 304 --layouts fwd dgrad --knob-sets gemm_stagger=200 gemm_stagger=400 gemm_stagger=800 > gpurun_out/r6_stagger.log 2>&1
cat gpurun_out/r6_stagger.log
