#!/bin/bash
# gpurun: attention PMC (fwd / dK-dV / dQ at B12 S2048 H32 D128 causal; one counter set per pass)
# then the serving-burst kernel trace (decode steps are graph replays).
set -o pipefail
mkdir -p gpurun_out/pmcattn3
export PYTHONPATH=$PWD
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
  for kind in ${KINDS:-fwd dkv dq}; do
    i=$((i+1))
    timeout -k 10 -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcattn3/$kind.$i -o run --output-format csv -- python3 $R/tools/attn_one.py $kind 5 12 2048 32 128 > $R/gpurun_out/pmcattn3/$kind.$i.log 2>&1 || { echo "fail $kind $set"; tail -5 $R/gpurun_out/pmcattn3/$kind.$i.log; exit 1; }
  done
done
cd $R && python tools/pmc_summary.py gpurun_out/pmcattn3 fa_ > gpurun_out/pmcattn3_summary.txt 2>&1; cat gpurun_out/pmcattn3_summary.txt
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/decprof3 -o run -- python3 -c "
import json, sys
sys.path.insert(0, '$R')
from llmctl.benchmarks.serving import run_serving_benchmark
print(json.dumps(run_serving_benchmark('gpt-7b', prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16, scheduler='prefill_first', max_batch_tokens=4096)))
" > $R/gpurun_out/decprof3.log 2>&1 || { tail -20 $R/gpurun_out/decprof3.log; exit 1; }
grep tpot $R/gpurun_out/decprof3.log | cut -c1-400
