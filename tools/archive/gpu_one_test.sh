set -o pipefail
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "side_stream" 2>&1 | tail -5
