#!/bin/bash
# gpurun: decode GEMM config sweep (skinny_linear_cfg incl. the multi-row-tile configs) vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u tools/skinny_sweep.py ${CFGS:-3,7,8,9,10,11,12,13,14} > gpurun_out/skinny_sweep.jsonl 2> gpurun_out/skinny_sweep.err || { tail -20 gpurun_out/skinny_sweep.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/skinny_sweep.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l)
    print(d['shape'], d['M'], d['best'], ' '.join(f"{k}={v['TBps']}" for k,v in d.items() if isinstance(v,dict)))
PY
