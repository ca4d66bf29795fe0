set -o pipefail
bash tools/gpu_attn.sh && SKIP_TESTS= bash tools/gpu_bench_ab.sh
