#!/bin/bash
# gpurun: full GPU test suite, then a two-ranks-on-one-GPU RCCL probe (informational).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 180 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1
echo "rccl probe rc=$?"
tail -15 gpurun_out/rccl_probe.log
