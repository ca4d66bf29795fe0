#!/bin/bash
# GPU call: micro-batch sweep of bench.py + one rocprofv3 kernel-stats profile.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
MBS=${MBS:-"8 12"}
for mb in $MBS; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 2 --micro-batch $mb > gpurun_out/bench_mb$mb.json 2> gpurun_out/bench_mb$mb.err || exit $?
  cat gpurun_out/bench_mb$mb.json
done
cd /tmp && export TMPDIR=/tmp
PMB=${PMB:-8}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --micro-batch $PMB > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || exit $?
ls -R $GRAFT_REPO_ROOT/gpurun_out/prof | head -20
