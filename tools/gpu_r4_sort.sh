# Round-4 sort check: the sort tests, then C3 / b1_merge / C2 timed on the
# new library, the round-3 library (build/base) and the wide-always variant
# (build/var_wide), one box; kernel stats of C3 and b1_merge on the new one.
#   bash tools/gpu_r4_sort.sh TAG
set -o pipefail
T=${1:-r4s}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "${KEXPR:-sort}" \
  tests/test_gpu_sort.py > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh ${T}_c3 python tools/bench_extra.py --workload c3 > gpurun_out/${T}_c3_sum.txt 2>&1 || exit 1
head -24 gpurun_out/${T}_c3_sum.txt
bash tools/gpu_prof.sh ${T}_b1m python tools/bench_extra.py --workload b1_merge --steps 2 > gpurun_out/${T}_b1m_sum.txt 2>&1 || exit 1
head -24 gpurun_out/${T}_b1m_sum.txt
bash tools/gpu_ab.sh ${T}_ab "" "${WORKS:-c3 b1_merge c2}" new build/base/liblime_amd.so ${VARS:-build/var_wide/liblime_amd.so}
