set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s22_tests.txt 2>&1
bash tools/ab.sh ab3 build/base/liblime_amd.so new
