# HBM bytes (FETCH_SIZE x2, WRITE_SIZE) and SQ issue / stall counters per
# kernel for one bench_extra workload, one rocprofv3 --pmc pass each.
#   bash tools/gpu_r4_pmc.sh TAG WORKLOAD
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-pmc}; W=${2:-c3}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_$C -o p -- python tools/bench_extra.py --workload $W --steps 1 --warmup 0 > gpurun_out/${T}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${T}_FETCH_SIZE gpurun_out/${T}_WRITE_SIZE > gpurun_out/${T}_bytes.txt
head -40 gpurun_out/${T}_bytes.txt
bash tools/gpu_pmc_sq.sh ${T} $W > /dev/null && head -60 gpurun_out/${T}_sq_summary.txt
