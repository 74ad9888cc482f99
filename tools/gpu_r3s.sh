# Round-3: rocPRIM sort bar, C3 kernel stats, then the 1e9-row / full-C5
# scale tests.  bash tools/gpu_r3s.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r3s}
step() {  # name timeout cmd...: stop the script on a fault / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/${T}_${name}.txt | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step rocprim_c2 120 ./bin/rocprim_sort_probe 100000000 0
step rocprim_c3 120 ./bin/rocprim_sort_probe 500000000 1
step c3_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3_stats -o run -- python tools/bench_extra.py --workload c3
python3 tools/kstats.py gpurun_out/${T}_c3_stats | head -16
step scale 1000 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_gpu_scale.py
