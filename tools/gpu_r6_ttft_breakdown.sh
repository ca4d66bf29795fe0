set -o pipefail
timeout -k 10 300 python -u tools/ttft_breakdown.py > gpurun_out/r6_ttft_breakdown.log 2>&1 && grep "^{" gpurun_out/r6_ttft_breakdown.log
