#!/bin/bash
# gpurun: streaming decode GEMM: decode kernel tests, bandwidth, decode step A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q -k "decode or skinny" --timeout 120 --timeout-method thread > gpurun_out/dstream_test.log 2>&1 || { tail -40 gpurun_out/dstream_test.log; exit 1; }
tail -2 gpurun_out/dstream_test.log
timeout -k 10 300 python -u tools/decode_gemm_bw.py --configs 25 > gpurun_out/dgemm.jsonl 2> gpurun_out/dgemm.err || { tail -20 gpurun_out/dgemm.err; exit 1; }
cat gpurun_out/dgemm.jsonl
for v in 1 0; do
  LLMCTL_KNOBS="decode_stream=$v" timeout -k 10 300 python -u tools/decode_host_breakdown.py > gpurun_out/serve_dec$v.json 2> gpurun_out/serve_dec$v.err || { tail -20 gpurun_out/serve_dec$v.err; exit 1; }
  echo "decode_stream=$v $(tail -1 gpurun_out/serve_dec$v.json)"
done
