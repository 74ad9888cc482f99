# bitset parity + C4 / C5 lines on the default build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-bc}
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_gpu_scale.py -k "bitset or c4 or c5 or complement or _and" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_c4.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/${T}_c4.txt
timeout -k 10 300 python bench.py --workload c5 --steps 5 --no-cpu-baseline > gpurun_out/${T}_c5.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/${T}_c5.txt | cut -c1-400
