#!/bin/bash
# GPU call: all GPU tests, smoke, kernel benches, serving benches, 7B training bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" | tee -a gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -m llmctl bench kernels --kv-cache --flash --rope > gpurun_out/bench_kernels.json 2> gpurun_out/bench_kernels.err || exit $?
timeout -k 10 400 python -c "
import json
from llmctl.benchmarks.serving import single_request_ttft, run_serving_benchmark
print(json.dumps(single_request_ttft('gpt-7b', 2048, 5)))
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16)))
" > gpurun_out/serve_bench.json 2> gpurun_out/serve_bench.err || exit $?
cat gpurun_out/serve_bench.json
