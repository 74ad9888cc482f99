# C4 kernel stats + the rocprofv3 trace (gaps between kernels)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-c4p}
bash tools/gpu_prof.sh ${T} python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_sum.txt 2>&1; rc=$?
head -30 gpurun_out/${T}_sum.txt; exit $rc
