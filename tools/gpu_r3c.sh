# Round-3: parity of the touched paths, C3 line, then PMC passes over the C2
# line (SQ issue/stall/LDS counters; HBM FETCH_SIZE / WRITE_SIZE, one pass
# each).  bash tools/gpu_r3c.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r3c}
step() {  # name timeout cmd...: stop the script on a fault / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/${T}_${name}.txt | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_parity.py -k "window_end or sort or bitset"
step c3 300 python tools/bench_extra.py --workload c3
P="bench.py --steps 1 --warmup 1 --no-cpu-baseline"
step sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/${T}_sq -o p -- python $P
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o p -- python $P
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o p -- python $P
python3 tools/pmc_summary.py gpurun_out/${T}_sq gpurun_out/${T}_fetch gpurun_out/${T}_write > gpurun_out/${T}_pmc_summary.txt
grep -E "local_small|k_scatter|k_prep|k_hist|k_merge|k_count|k_windows" gpurun_out/${T}_pmc_summary.txt | head -80
