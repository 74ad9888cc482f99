set -e
mkdir -p gpurun_out
timeout -k 10 120 ./bin/alloc_probe > gpurun_out/s23_alloc.jsonl 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s23_tests.txt 2>&1
bash tools/ab.sh ab4 build/base/liblime_amd.so new
timeout -k 10 120 ./bin/alloc_probe > gpurun_out/s23_alloc2.jsonl 2>&1
