# HBM bytes per kernel: one rocprofv3 --pmc pass per counter (MI355X_MICROARCH.md)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-pmc}; shift
W=${1:-c5}; shift
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_$C -o p -- python bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${T}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${T}_FETCH_SIZE gpurun_out/${T}_WRITE_SIZE
