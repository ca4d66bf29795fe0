#!/bin/bash
# Round 6: long-context measurements on one MI355X -- GPT-7B training at 32k tokens per step with
# seq 8k / 16k / 32k (flash attention fwd / bwd at long S), and single-prompt TTFT at 8k / 16k / 32k
# prompts (chunked prefill: 8,192-token chunks, later chunks through the paged prefill kernel).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
: > gpurun_out/longctx.log
for sm in "8192 4" "16384 2" "32768 1"; do
  set -- $sm
  timeout -k 10 400 python bench.py --seq-len $1 --micro-batch $2 --steps 4 --warmup 2 2> gpurun_out/longctx_train_$1.err \
    | grep '^{' >> gpurun_out/longctx.log || { tail -20 gpurun_out/longctx_train_$1.err; exit 1; }
done
for n in 8192 16384 32768; do
  timeout -k 10 300 python tools/ttft_bench.py --prompt-length $n --repeats 3 2> gpurun_out/longctx_ttft_$n.err \
    | grep '^{' >> gpurun_out/longctx.log || { tail -20 gpurun_out/longctx_ttft_$n.err; exit 1; }
done
