set -o pipefail
mkdir -p gpurun_out
T=${1:-r3h}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_sort.py tests/test_gpu_parity.py -k "strands or same_start or sort or subtract" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/bench_extra.py --workload subtract > gpurun_out/${T}_sub.txt 2>&1; tail -1 gpurun_out/${T}_sub.txt | cut -c1-400
bash tools/gpu_pmc_sq.sh ${T} c2 2>&1 | grep -E "local_small|scatter|k_prep|k_hist" | head -40
