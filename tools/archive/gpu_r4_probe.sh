#!/bin/bash
# gpurun: 4-wave GEMM bottleneck probes (no memory traffic / no barriers / no epilogue)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/gemm_probe.py --config 904 --probes 0 1 32 64 16 48 80 > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
