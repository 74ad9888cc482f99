set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s20_tests.txt 2>&1
timeout -k 10 300 python tools/bench_extra.py --workload bed > gpurun_out/s20_bed.txt 2>&1
