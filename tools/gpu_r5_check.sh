# Round-5 check on one box: GPU tests (KEXPR over the -m gpu suite), then
# kernel stats of bench_extra workloads (WORKS) on the in-tree library.
#   KEXPR=... WORKS="c3 b1_merge" bash tools/gpu_r5_check.sh TAG
set -o pipefail
T=${1:-r5c}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "$KEXPR" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
  tail -2 gpurun_out/${T}_tests.txt
fi
for W in $WORKS; do
  bash tools/gpu_prof.sh ${T}_$W python tools/bench_extra.py --workload $W > gpurun_out/${T}_${W}_sum.txt || exit 1
  grep '^{' gpurun_out/${T}_${W}_prof.txt | tail -1 | cut -c1-400
  head -12 gpurun_out/${T}_${W}_sum.txt
done
