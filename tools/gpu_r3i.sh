# C4 kernel stats + C3 merge SQ counters.  bash tools/gpu_r3i.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r3i}
bash tools/gpu_prof.sh ${T}_c4 python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_c4sum.txt 2>&1 || { tail -5 gpurun_out/${T}_c4sum.txt; exit 1; }
head -24 gpurun_out/${T}_c4sum.txt
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/${T}_sq -o p -- python tools/bench_extra.py --workload c3 --steps 1 --warmup 1 > gpurun_out/${T}_sq.log 2>&1 || { tail -5 gpurun_out/${T}_sq.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/${T}_sq > gpurun_out/${T}_sq_summary.txt
grep -E "merge_scan2|k_scatter|k_prep|k_hist" gpurun_out/${T}_sq_summary.txt
