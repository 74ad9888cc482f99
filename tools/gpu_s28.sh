set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "sort or merge or scaled or intersect_parity or stranded" > gpurun_out/s28_tests.txt 2>&1
bash tools/ab.sh ab6 build/base/liblime_amd.so new
