# merge kernel A/B: parity of the merge paths, then C3 and C2 lines with the
# new k_merge_scan2 and with LIME_MERGE_V1=1 (the transposing kernel)
set -o pipefail
mkdir -p gpurun_out
T=${1:-mab}
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -k "merge or c3 or cluster or subtract or c2_full or sharded" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for V in "" 1; do
  timeout -k 10 300 env LIME_MERGE_V1=$V python tools/bench_extra.py --workload c3 > gpurun_out/${T}_c3_v$V.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_c3_v$V.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c3 v1=$V', d['breakdown_ms'], d['roofline']['frac'])"
done
done
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/${T}_c2.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/${T}_c2.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c2', d['breakdown_ms'], d['ms_per_step'])"
