# Round-5 verification on one box: the whole GPU suite (scale tests
# included), smoke, the default bench line (CPU baseline included) and the C5
# line, then rocprofv3 kernel stats of the default line and of the C5, C3 and
# 1e9-subtract workloads.  bash tools/gpu_r5_final.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5f}
step() {  # name timeout cmd...: stop the script on a fault / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/${T}_${name}.txt | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -z "$NOSUITE" ]; then
  step suite 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_c2 500 python bench.py
step bench_c5 300 python bench.py --workload c5
step c2_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c2_stats -o run -- python bench.py --steps 5 --no-cpu-baseline
for W in c5 c3 sub; do
  step ${W}_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_${W}_stats -o run -- python bench.py --workload $W --steps 5 --no-cpu-baseline
done
