set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s11_tests.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s11_prof -o run -- python bench.py --steps 5 --no-cpu-baseline > gpurun_out/s11_bench.txt 2>&1
timeout -k 10 200 python tools/bench_extra.py --workload c3 > gpurun_out/s11_c3.txt 2>&1
