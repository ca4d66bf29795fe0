#!/bin/bash
# gpurun: the driver's multi-GPU launch form with one rank (RCCL world 1 through torchrun)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 4 --warmup 2 > gpurun_out/tr1.json 2> gpurun_out/tr1.err || { tail -30 gpurun_out/tr1.err; exit 1; }
cat gpurun_out/tr1.json
grep -iE "layout|zero|warn" gpurun_out/tr1.err | head -5
