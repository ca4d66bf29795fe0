#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --micro-batch 8 > gpurun_out/bench_sink_mb8.json 2> gpurun_out/bench_sink_mb8.err || exit $?
cat gpurun_out/bench_sink_mb8.json
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_results%d.csv
timeout -k 10 600 python bench.py --steps 4 --warmup 3 --micro-batch 8 > gpurun_out/bench_tuned_mb8.json 2> gpurun_out/bench_tuned_mb8.err || exit $?
cat gpurun_out/bench_tuned_mb8.json
ls gpurun_out/
