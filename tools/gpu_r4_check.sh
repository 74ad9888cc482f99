# Round-4 targeted GPU check: a pytest -k selection (KEXPR), then optional
# bench_extra workloads (WORKS) with kernel stats.   bash tools/gpu_r4_check.sh TAG
set -o pipefail
T=${1:-r4c}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu \
    -k "$KEXPR" ${TFILES:-tests} > gpurun_out/${T}_tests.txt 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${T}_tests.txt | tail -30; [ $rc -eq 0 ] || exit $rc
fi
for W in $WORKS; do
  bash tools/gpu_prof.sh ${T}_$W python tools/bench_extra.py --workload $W > gpurun_out/${T}_${W}_sum.txt 2>&1 || { tail -20 gpurun_out/${T}_${W}_sum.txt; exit 1; }
  head -22 gpurun_out/${T}_${W}_sum.txt
  grep -h '^{' gpurun_out/${T}_${W}_prof.txt | cut -c1-600
done
