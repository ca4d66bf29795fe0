#!/bin/bash
# Round 6 final check: full GPU suite + smoke + bench, then a rocprofv3 --stats profile of the default bench.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_full_check.sh || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bench_prof_r6 -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/bench_prof_r6.log 2>&1
