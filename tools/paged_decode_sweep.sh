# Paged decode attention over serving shapes and context splits (0 = the auto heuristic);
# output: gpurun_out/pd_sweep.log (JSON lines from tools/paged_decode_bw.py)
set -o pipefail
T="timeout -k 10 150 python tools/paged_decode_bw.py --contig --rounds 2"
$T --splits 0 1 2 4 > gpurun_out/pd_sweep.log 2>&1 &&
$T --Hq 32 --Hkv 8 --splits 0 1 2 4 8 >> gpurun_out/pd_sweep.log 2>&1 &&
$T --N 64 --ctx 1024 --splits 0 1 2 >> gpurun_out/pd_sweep.log 2>&1 &&
$T --N 1 --ctx 8192 --Hq 64 --Hkv 8 --splits 0 16 32 64 >> gpurun_out/pd_sweep.log 2>&1 &&
$T --N 1 --ctx 8192 --Hq 32 --Hkv 32 --splits 0 8 16 32 >> gpurun_out/pd_sweep.log 2>&1 &&
$T --N 4 --ctx 4096 --splits 0 2 4 8 >> gpurun_out/pd_sweep.log 2>&1
