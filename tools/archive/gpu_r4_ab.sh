#!/bin/bash
# gpurun: interleaved GPT-7B bench A/B of performance-knob sets ($A_KNOBS vs $B_KNOBS, LLMCTL_KNOBS
# syntax), ROUNDS rounds (default 2), optional pytest -k filter $TESTS run first.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/kernels -x -q --timeout 120 --timeout-method thread -k "$TESTS" > gpurun_out/ab_test.log 2>&1; rc=$?
  tail -1 gpurun_out/ab_test.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/ab_test.log | head; exit $rc; }
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  for k in "$A_KNOBS" "$B_KNOBS"; do
    LLMCTL_KNOBS="$k" timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "[$k] $(tail -1 gpurun_out/ab.log | cut -c1-170)"
  done
done
