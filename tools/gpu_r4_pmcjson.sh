# HBM traffic JSON for bench.py's roofline "traffic" (profiles/pmc_c2.json,
# profiles/pmc_c5.json): FETCH_SIZE and WRITE_SIZE passes of the bench command
# itself, one rocprofv3 --pmc run each, then tools/pmc_json.py.
#   bash tools/gpu_r4_pmcjson.sh TAG COMMIT
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-pmcj}; SHA=${2:-unknown}
c2="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops"
c5="python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline"
for W in c2 c5; do
  cmd=${!W}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_${W}_$C -o p -- $cmd > gpurun_out/${T}_${W}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_${W}_$C.log; exit 1; }
  done
done
python tools/pmc_json.py gpurun_out/${T}_pmc_c2.json gpurun_out/${T}_c2_FETCH_SIZE gpurun_out/${T}_c2_WRITE_SIZE --commit "$SHA" --cmd "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- $c2" --key "k_fill<1, false, false>" || exit 1
python tools/pmc_json.py gpurun_out/${T}_pmc_c5.json gpurun_out/${T}_c5_FETCH_SIZE gpurun_out/${T}_c5_WRITE_SIZE --commit "$SHA" --cmd "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- $c5" --steps 3 --exclude k_uniform || exit 1
python tools/pmc_summary.py gpurun_out/${T}_c5_FETCH_SIZE gpurun_out/${T}_c5_WRITE_SIZE > gpurun_out/${T}_c5_bytes.txt && head -30 gpurun_out/${T}_c5_bytes.txt
