#!/bin/bash
# gpurun: prefill-step host breakdown of the 16 x 2048 burst at 2048 / 4096 / 8192-token budgets
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u tools/prefill_host_breakdown.py 2048 4096 8192 > gpurun_out/pf_host.jsonl 2> gpurun_out/pf_host.err || { tail -20 gpurun_out/pf_host.err; exit 1; }
cat gpurun_out/pf_host.jsonl
