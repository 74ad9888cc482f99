set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s16_tests.txt 2>&1
bash tools/ab.sh ab2 build/base/liblime_amd.so new
