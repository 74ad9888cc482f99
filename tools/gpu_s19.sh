set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s19_tests.txt 2>&1
