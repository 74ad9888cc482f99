# A/B of the fill finding the owners' ranges itself (LIME_FILL_SEARCH=1, the
# default build) against k_count writing them (build/var_nosearch): intersect
# parity, then C2 and the sparse 1e9-row pairwise line, alternated.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-fs}
V=build/var_nosearch/liblime_amd.so
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_gpu_threads.py -k "not c3_full and not c5 and not c4 and not bitset" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in "" $V; do
    timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python bench.py --steps 5 --no-cpu-baseline > gpurun_out/${T}_c2_$r${L:+_v}.txt 2>&1 || exit 1
    grep -h '^{' gpurun_out/${T}_c2_$r${L:+_v}.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c2 var=${L:+nosearch}', d['ms_per_step'], d['breakdown_ms'])"
  done
done
for L in "" $V; do
  timeout -k 10 400 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload b1_pair --steps 1 > gpurun_out/${T}_b1_${L:+v}.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_b1_${L:+v}.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); b=d['breakdown_ms']; print('b1_pair var=${L:+nosearch}', {k: b[k] for k in ('sort_ms','count_ms','fill_ms')})"
done
bash tools/gpu_prof.sh ${T}_c2 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/${T}_kstats.txt; head -16 gpurun_out/${T}_kstats.txt
