set -o pipefail
bash tools/gpu_attn.sh && bash tools/gpu_ttft.sh
