# C4 kernel stats and the last step's dispatch timeline (gaps = host syncs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-c4t}
bash tools/gpu_prof.sh ${T} python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_sum.txt 2>&1 || exit 1
head -30 gpurun_out/${T}_sum.txt
python3 tools/trace_tail.py gpurun_out/${T}_stats 45 > gpurun_out/${T}_tail.txt
cat gpurun_out/${T}_tail.txt
