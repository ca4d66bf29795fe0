#!/bin/bash
# gpurun: in-GEMM decode finalize: decode kernel tests, then the serving measurements
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q -k "decode" --timeout 120 --timeout-method thread > gpurun_out/decfin_test.log 2>&1 || { tail -40 gpurun_out/decfin_test.log; exit 1; }
tail -2 gpurun_out/decfin_test.log
for fin in ${FINS:-15 7 3 0}; do
  LLMCTL_KNOBS="decode_fin=$fin" timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/serve_dec$fin.json 2> gpurun_out/serve_dec$fin.err || { tail -20 gpurun_out/serve_dec$fin.err; exit 1; }
  echo "decode_fin=$fin $(tail -1 gpurun_out/serve_dec$fin.json)"
done
