# Round-3 check of the current tree on one GPU: GPU suite (no 1e9-row tests),
# smoke, C2/C5 bench lines, C3/C4/subtract lines, rocprofv3 kernel stats of
# the C2 line.  bash tools/gpu_r3v.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r3v}
step() {  # name timeout cmd...: stop the script on a fault / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/${T}_${name}.txt | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step suite 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests --ignore tests/test_gpu_scale.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 400 python bench.py --steps 10 --warmup 2
step bench_c5 300 python bench.py --workload c5 --no-cpu-baseline
for W in c3 c4 subtract; do step $W 300 python tools/bench_extra.py --workload $W; done
step c2_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c2_stats -o run -- python bench.py --steps 5 --no-cpu-baseline
python3 tools/kstats.py gpurun_out/${T}_c2_stats | head -30
