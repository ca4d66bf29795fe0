#!/bin/bash
# gpurun: final state of round 4 -- smoke + whole GPU suite + driver-default bench, then the
# rocprofv3 kernel stats of the default step
set -o pipefail
bash tools/gpu_r4_full.sh && ARMS=";" TOP=30 bash tools/gpu_r4_prof2.sh
