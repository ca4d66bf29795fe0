#!/bin/bash
# gpurun: single-request TTFT, then a rocprofv3 kernel-stats pass over it.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/ttft_bench.py ${TTFT_ARGS} > gpurun_out/ttft.json 2> gpurun_out/ttft.err || { tail -20 gpurun_out/ttft.err; exit 1; }
cat gpurun_out/ttft.json
if [ -n "$PROF" ]; then
  R=$PWD
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ttft -o run --output-format csv -- python3 $R/tools/ttft_bench.py --repeats 3 > $R/gpurun_out/prof_ttft.log 2>&1 || { tail -20 $R/gpurun_out/prof_ttft.log; exit 1; }
  echo prof ok
fi
