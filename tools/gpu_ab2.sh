# A/B after the window / look-back changes: parity of the touched paths, C3
# merge with the 4-window look-back and with LIME_MERGE_LB1=1, C2 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-ab2}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_closest.py tests/test_gpu_threads.py -k "not c3_full and not c5 and not c4" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for V in "" 1; do
  timeout -k 10 300 env LIME_MERGE_LB1=$V python tools/bench_extra.py --workload c3 > gpurun_out/${T}_c3_v$V.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_c3_v$V.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c3 lb1=$V', d['breakdown_ms'], d['roofline']['frac'])"
done
done
bash tools/gpu_prof.sh ${T}_c2 python bench.py --steps 5 --no-cpu-baseline | head -14
grep -h '^{' gpurun_out/${T}_c2_prof.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c2', d['breakdown_ms'], d['ms_per_step'])"
