set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s1_tests.txt 2>&1
timeout -k 10 120 ./bin/bw_probe > gpurun_out/s1_probe.jsonl 2>&1
timeout -k 10 300 python bench.py > gpurun_out/s1_bench.txt 2>&1
