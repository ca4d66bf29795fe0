set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp configs/tuning/tunableop_mi355x_gpt7b.csv gpurun_out/tun2.csv
timeout -k 10 700 python -u tools/gemm_tunable.py --tokens 24576 --ops wgrad,wgradT,transpose --skip-rocblas --append --csv gpurun_out/tun2.csv > gpurun_out/tune_wgradT.log 2>&1; rc=$?; grep -v "^tuned\|amdgpu" gpurun_out/tune_wgradT.log | tail -30; exit $rc
