# A/B of the direct per-bin paint for sparse row sets (default build) against
# the split + per-tile paint (build/var_nodirect): bitset parity, C4 and C5
# alternated, then C4's dispatch timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-dp}
V=build/var_nodirect/liblime_amd.so
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -k "bitset or c4 or c5 or complement or _and" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in "" $V; do
    timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_c4_$r${L:+_v}.txt 2>&1 || exit 1
    grep -h '^{' gpurun_out/${T}_c4_$r${L:+_v}.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c4 var=${L:+nodirect}', d['ms_per_step'], d['breakdown_ms'])"
  done
done
timeout -k 10 300 python bench.py --workload c5 --steps 5 --no-cpu-baseline > gpurun_out/${T}_c5.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/${T}_c5.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c5', d['ms_per_step'])"
bash tools/gpu_prof.sh ${T}_c4 python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_kstats.txt || exit 1
head -24 gpurun_out/${T}_kstats.txt
python3 tools/trace_tail.py gpurun_out/${T}_c4_stats 40 > gpurun_out/${T}_tail.txt
cat gpurun_out/${T}_tail.txt
