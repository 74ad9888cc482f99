set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r2p
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "subtract" tests/test_gpu_threads.py > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_sub -o run -- python tools/bench_extra.py --workload subtract --steps 1 --warmup 1 > gpurun_out/${T}_sub.txt 2>&1 || exit 1
find gpurun_out/${T}_sub -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_sub_kernel_stats.csv \;
