# Round-3 final verification, part 1: the whole GPU suite (scale tests
# included), smoke, the default bench line (CPU baseline included) and the C5
# line, rocprofv3 kernel stats of both.  bash tools/gpu_verify3.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-v3}
step() {  # name timeout cmd...: stop the script on a fault / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/${T}_${name}.txt | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step suite 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 400 python bench.py
step bench_c5 300 python bench.py --workload c5
step c2_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c2_stats -o run -- python bench.py --steps 5 --no-cpu-baseline
step c5_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c5_stats -o run -- python bench.py --workload c5 --steps 5 --no-cpu-baseline
