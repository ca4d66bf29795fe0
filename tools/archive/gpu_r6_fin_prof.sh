#!/bin/bash
# Round 6: per-kernel decode-step stats with the finalize inside the GEMM (decode_fin=1) vs separate (0).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1; do
  LLMCTL_KNOBS="decode_fin=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/finprof_$v -o run -- \
    python3 $R/tools/decode_host_breakdown.py --tokens 48 > $R/gpurun_out/finprof_$v.log 2>&1 || exit 1
done
