set -o pipefail
timeout -k 10 400 python -u tools/gemm4w_bench.py --configs 304 --layouts fwd dgrad --knob-sets gemm_nt_c=1 > gpurun_out/r6_ntc.log 2>&1
cat gpurun_out/r6_ntc.log
