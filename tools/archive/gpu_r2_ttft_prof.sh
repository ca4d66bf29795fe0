#!/bin/bash
# gpurun: kernel stats of isolated 2k-token prefills (TTFT path), gemm64 forward on / off
mkdir -p gpurun_out
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  LLMCTL_FWD64=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ttftprof$v -o run --output-format csv -- python3 $R/tools/ttft_bench.py --repeats 5 > $R/gpurun_out/ttftprof$v.log 2>&1 || { tail -20 $R/gpurun_out/ttftprof$v.log; exit 1; }
  grep ttft_p50 $R/gpurun_out/ttftprof$v.log
done
