set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 200 python tools/attn_ablate.py > gpurun_out/attn_ablate.log 2>&1; rc=$?; cat gpurun_out/attn_ablate.log; exit $rc
