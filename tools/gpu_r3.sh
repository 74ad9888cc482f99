# Round-3 GPU check: new sort tests, C2/C3 bench lines, rocPRIM bar, the GPU
# suite and the full-scale parity tests.  bash tools/gpu_r3.sh TAG
set -o pipefail
mkdir -p gpurun_out
T=${1:-r3}
step() {  # name timeout cmd...: stop the script on a fault / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/${T}_${name}.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
step sort 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_sort.py
step bench_c2 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline
step c3 300 python tools/bench_extra.py --workload c3
[ -x bin/rocprim_sort_probe ] && step rocprim 200 ./bin/rocprim_sort_probe 100000000 0
step suite 600 python -u -m pytest -q -x --timeout 400 --timeout-method thread -m gpu tests --ignore tests/test_gpu_scale.py --ignore tests/test_gpu_sort.py
step scale 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_scale.py
