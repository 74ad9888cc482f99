set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r2k
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
LIME_BIN_DIRECT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py::test_c5_eight_way_and_density > gpurun_out/${T}_tests2.txt 2>&1 || { tail -40 gpurun_out/${T}_tests2.txt; exit 1; }
for v in 0 1; do
LIME_BIN_DIRECT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c5_$v -o run -- python tools/bench_extra.py --workload c5 --steps 2 --warmup 1 > gpurun_out/${T}_c5p_$v.txt 2>&1 || exit 1
find gpurun_out/${T}_c5_$v -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_c5_kernel_stats_$v.csv \;
done
