set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tl -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/tl_bench.log 2>&1 &&
python3 tools/step_timeline.py gpurun_out/tl > gpurun_out/tl_summary.txt 2>&1 &&
cat gpurun_out/tl_summary.txt
