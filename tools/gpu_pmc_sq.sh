# Issue / stall / LDS counters per kernel, one rocprofv3 --pmc pass (8 SQ
# counters, the block's limit):  bash tools/gpu_pmc_sq.sh TAG WORKLOAD [bench args]
# (WORKLOAD c2 / c5: bench.py; others: tools/bench_extra.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-sq}; shift
W=${1:-c5}; shift
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
case $W in
  c2|c5) P="bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline" ;;
  *) P="tools/bench_extra.py --workload $W --steps 1 --warmup 1" ;;
esac
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_sq -o p -- python $P "$@" > gpurun_out/${T}_sq.log 2>&1 || { tail -5 gpurun_out/${T}_sq.log; exit 1; }
python tools/pmc_summary.py gpurun_out/${T}_sq > gpurun_out/${T}_sq_summary.txt
head -60 gpurun_out/${T}_sq_summary.txt
