# Round-5 sort check: the sort GPU tests on the new library, then the C3 /
# 1e9 merge-side / C2 lines on the new and a base library (same box), then
# kernel stats of the C3 line on the new one.
#   bash tools/gpu_r5_sort.sh TAG BASELIB [KEXPR]
set -o pipefail
T=$1; BASE=$2; K=${3:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "$K" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
  tail -3 gpurun_out/${T}_tests.txt
fi
bash tools/gpu_ab.sh ${T}ab "" "c3 b1_merge c2" new $BASE || exit 1
bash tools/gpu_prof.sh ${T}c3 python tools/bench_extra.py --workload c3 || exit 1
if [ -n "$PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_$C -o p -- python tools/bench_extra.py --workload $PMC --steps 1 --warmup 0 > gpurun_out/${T}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_$C.log; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/${T}_FETCH_SIZE gpurun_out/${T}_WRITE_SIZE > gpurun_out/${T}_bytes.txt
  head -24 gpurun_out/${T}_bytes.txt
fi
