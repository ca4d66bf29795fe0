#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
i=10
for extra in "--pp 2 --zero 0" "--cp 2 --zero 0" "--cp 2 --cp-mode ring --zero 0" "--model tiny-moe --ep 2 --seq-len 256 --zero 1" "--zero 3"; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29650+i)) \
    bench.py --gpus 2 --model gpt-125m --seq-len 1024 --micro-batch 4 --steps 3 --warmup 1 --device cuda:0 --backend gloo $extra \
    > gpurun_out/multirank_$i.json 2> gpurun_out/multirank_$i.err
  rc=$?
  echo "[$extra] rc=$rc $(grep -h '^{' gpurun_out/multirank_$i.json | cut -c1-60) $(grep -h '"parallelism"' gpurun_out/multirank_$i.json | grep -o '"parallelism": "[^"]*"\|"final_loss": [0-9.]*' | tr '\n' ' ')"
  [ $rc -ne 0 ] && tail -4 gpurun_out/multirank_$i.err
  i=$((i+1))
done
exit 0
