# sort tests, then the C3 line with kernel stats.  bash tools/gpu_c3.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-c3}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_sort.py > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh ${T}_c3 python tools/bench_extra.py --workload c3 > gpurun_out/${T}_sum.txt 2>&1; rc=$?
head -16 gpurun_out/${T}_sum.txt
grep -h '^{' gpurun_out/${T}_c3_prof.txt | cut -c1-400
exit $rc
