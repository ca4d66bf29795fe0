#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/debug_p3b.py 8 > gpurun_out/dbg.log 2>&1 || { tail -20 gpurun_out/dbg.log; exit 1; }
cat gpurun_out/dbg.log
