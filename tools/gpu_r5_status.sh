# Round-5 status sweep on one box: kernel stats of the bench_extra lines
# (WORKS), then FETCH / WRITE PMC passes of the C3 line (sort bytes per row).
#   WORKS="c3 b1_merge c4 c5" bash tools/gpu_r5_status.sh TAG
set -o pipefail
T=${1:-r5s}
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in ${WORKS:-c3 b1_merge c4 c5}; do
  bash tools/gpu_prof.sh ${T}_$W python tools/bench_extra.py --workload $W > gpurun_out/${T}_${W}_sum.txt || exit 1
  echo "== $W: $(grep '^{' gpurun_out/${T}_${W}_prof.txt | tail -1 | cut -c1-600)"
  head -14 gpurun_out/${T}_${W}_sum.txt
done
if [ -n "$PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_$C -o p -- python tools/bench_extra.py --workload $PMC --steps 1 --warmup 0 > gpurun_out/${T}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_$C.log; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/${T}_FETCH_SIZE gpurun_out/${T}_WRITE_SIZE > gpurun_out/${T}_bytes.txt
  head -30 gpurun_out/${T}_bytes.txt
fi
