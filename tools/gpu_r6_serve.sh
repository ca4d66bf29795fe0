# round 6: serving GPU tests (TP async pipeline, fp8 large batch) + TP=2 GPT-7B decode timing
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/kernels/test_serving_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r6_serve_tests.log 2>&1 &&
tail -3 gpurun_out/r6_serve_tests.log && grep "TP=" gpurun_out/r6_serve_tests.log &&
timeout -k 10 500 python -u tools/tp_decode_timing.py --world 2 --model gpt-7b --batch 16 --prompt 512 --tokens 64 > gpurun_out/r6_tp_decode.log 2>&1 &&
cat gpurun_out/r6_tp_decode.log | grep '^{'
