#!/bin/bash
# gpurun: two-rank PP with a tied LM head (gpt-125m, ranks share cuda:0 over gloo), then the
# round-end checks (smoke, GPU tests, 1-GPU bench, rocprofv3 kernel stats).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29711 \
  bench.py --gpus 2 --model gpt-125m --seq-len 1024 --micro-batch 4 --steps 3 --warmup 1 --device cuda:0 --backend gloo --pp 2 --zero 0 \
  > gpurun_out/pp_tied.json 2> gpurun_out/pp_tied.err || { grep -E "Error|error" gpurun_out/pp_tied.err | head -20; exit 1; }
grep '^{' gpurun_out/pp_tied.json | cut -c1-400
bash tools/gpu_final.sh
