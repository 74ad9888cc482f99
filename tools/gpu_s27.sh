set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s27_tests.txt 2>&1
bash tools/ab.sh ab5 build/base/liblime_amd.so new
