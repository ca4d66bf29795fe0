# GPT-7B serving burst (16 x 2048-token prompts -> 128 tokens, prefill_first, 4096-token budget): bf16, fp8 KV cache,
# fp8 KV cache + fp8 decode weights; plus the single-prompt TTFT.  JSON lines in gpurun_out/e2e_burst.log
set -o pipefail
: > gpurun_out/e2e_burst.log
for cfg in "auto auto" "fp8 auto" "fp8 fp8"; do
  set -- $cfg
  timeout -k 10 300 python -c "
import json
from llmctl.benchmarks.serving import run_serving_benchmark
r = run_serving_benchmark(model='gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                          scheduler='prefill_first', kv_cache_dtype='$1', weight_dtype='$2')
r['data'] = 'synthetic prompts, random-init weights'
print(json.dumps(r))
" 2>&1 | grep '^{' >> gpurun_out/e2e_burst.log || exit 1
done
timeout -k 10 300 python tools/ttft_bench.py 2>&1 | grep '^{' >> gpurun_out/e2e_burst.log
