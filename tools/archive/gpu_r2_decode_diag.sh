#!/bin/bash
# gpurun: host-phase breakdown of decode steps, then kernel stats of the 16 x 2048 -> 128 serving burst
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/dec_host.json 2> gpurun_out/dec_host.err || { tail -20 gpurun_out/dec_host.err; exit 1; }
cat gpurun_out/dec_host.json
bash tools/gpu_r2_decode_prof.sh
