set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r2q
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/${T}_tests.txt 2>&1 || { tail -60 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
