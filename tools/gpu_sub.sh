# subtract check: subtract parity tests (small, megabase, stress, ties,
# sharded), the full-size C2 and 1e9-row subtract tests, then the subtract
# and b1_pair lines with kernel stats.  bash tools/gpu_sub.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-sub}
timeout -k 10 700 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_gpu_scale.py tests/test_gpu_threads.py -k "subtract or sub_ or c1_cli" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_extra.py --workload subtract > gpurun_out/${T}_subtract.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/${T}_subtract.txt | cut -c1-420
bash tools/gpu_prof.sh ${T}_b1 python tools/bench_extra.py --workload b1_pair --steps 2 --warmup 1 > gpurun_out/${T}_b1sum.txt 2>&1; rc=$?
head -12 gpurun_out/${T}_b1sum.txt
grep -h '^{' gpurun_out/${T}_b1_prof.txt | cut -c1-600
exit $rc
