# SQ issue / stall / LDS counters of one bench_extra workload per library
# variant (one rocprofv3 --pmc pass each):
#   bash tools/gpu_sqvar.sh TAG WORKLOAD "KERNEL_REGEX" lib1 lib2 ...   (lib "new" = in-tree)
set -o pipefail
T=$1; W=$2; K=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${SQC:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS"}
for lib in "$@"; do
  unset LIME_AMD_LIB_VARIANT
  [ "$lib" != new ] && export LIME_AMD_LIB_VARIANT=$PWD/$lib
  tag=${T}_$(echo $lib | tr '/.' '__')
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${tag}_sq -o p -- python tools/bench_extra.py --workload $W --steps 1 --warmup 0 > gpurun_out/${tag}_sq.log 2>&1 || { tail -5 gpurun_out/${tag}_sq.log; exit 1; }
  echo "== $lib"
  python3 tools/pmc_summary.py gpurun_out/${tag}_sq | grep -E "$K"
done
