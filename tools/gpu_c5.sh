# bitset path check: the bitset parity tests (C4 / C5 / sharded included),
# then the C5 and C4 lines with kernel stats.  bash tools/gpu_c5.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-c5}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -k "bitset or c4 or c5 or sharded or complement or window_end" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh ${T}_c5 python bench.py --workload c5 --steps 5 --no-cpu-baseline | head -16
grep -h '^{' gpurun_out/${T}_c5_prof.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c5', d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python tools/bench_extra.py --workload c4 > gpurun_out/${T}_c4.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/${T}_c4.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c4', d['ms_per_step'], d['breakdown_ms'])"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/${T}_sq -o p -- python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_sq.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/${T}_sq > gpurun_out/${T}_sq_summary.txt
grep -E "bin_write|bin_split|bin_count|paint_and" gpurun_out/${T}_sq_summary.txt
