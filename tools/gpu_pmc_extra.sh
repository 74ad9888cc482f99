# HBM bytes per kernel for a tools/bench_extra.py workload (one --pmc pass per counter)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-pmcx}; W=${2:-closest}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_$C -o p -- python tools/bench_extra.py --workload $W --steps 1 --warmup 0 > gpurun_out/${T}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${T}_FETCH_SIZE gpurun_out/${T}_WRITE_SIZE | head -40
