# Round-end style check on one GPU: the whole GPU test suite (one process), smoke(), and a short
# default bench; logs under gpurun_out/.  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu_tests.log 2>&1 &&
tail -3 gpurun_out/full_gpu_tests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1 &&
tail -1 gpurun_out/full_smoke.log &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/full_bench.log 2>&1 &&
grep '^{' gpurun_out/full_bench.log
