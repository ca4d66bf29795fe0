#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/decode_exec_timing.py > gpurun_out/replay.json 2> gpurun_out/replay.err || { tail -20 gpurun_out/replay.err; exit 1; }
cat gpurun_out/replay.json
