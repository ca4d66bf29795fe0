#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 200 python -u tools/debug_dstream.py > gpurun_out/dbg2.log 2>&1 || { tail -20 gpurun_out/dbg2.log; exit 1; }
cat gpurun_out/dbg2.log
