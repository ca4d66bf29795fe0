#!/bin/bash
# gpurun: multi-rank GPU code paths on a one-GPU box — 2 ranks share cuda:0 over gloo (RCCL refuses
# two ranks on one device): DP ZeRO-0/1, TP=2; llama-style model small enough for two copies.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
i=0
for extra in ${CONFIGS:-"--zero 1" "--zero 0" "--tp 2 --zero 0" "--zero 2"}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29650+i)) \
    bench.py --gpus 2 --model ${MODEL:-gpt-125m} --seq-len 1024 --micro-batch 4 --steps 3 --warmup 1 --device cuda:0 --backend gloo $extra \
    > gpurun_out/multirank_$i.json 2> gpurun_out/multirank_$i.err || { tail -30 gpurun_out/multirank_$i.err; exit 1; }
  echo "[$extra] $(cat gpurun_out/multirank_$i.json)"
  i=$((i+1))
done
