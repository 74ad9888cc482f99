set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bitset or sort or merge or scaled" > gpurun_out/s29_tests.txt 2>&1
timeout -k 10 300 python tools/bench_extra.py --workload c4 > gpurun_out/s29_c4.txt 2>&1
timeout -k 10 300 python tools/bench_extra.py --workload c5 > gpurun_out/s29_c5.txt 2>&1
