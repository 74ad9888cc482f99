# C4 / C5 with the extraction tile geometry varied (build/var_*), after the
# bitset parity tests on the default build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-ev}
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -k "bitset or c4 or c5 or complement or _and" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in "" build/var_w8/liblime_amd.so build/var_nt512/liblime_amd.so build/var_w32/liblime_amd.so; do
    timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_c4.txt 2>&1 || exit 1
    grep -h '^{' gpurun_out/${T}_c4.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c4 var=$L', round(d['ms_per_step'],4), d['breakdown_ms'])"
  done
done
for L in "" build/var_w8/liblime_amd.so build/var_nt512/liblime_amd.so build/var_w32/liblime_amd.so; do
  timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python bench.py --workload c5 --steps 5 --no-cpu-baseline > gpurun_out/${T}_c5.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_c5.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c5 var=$L', d['ms_per_step'], d.get('breakdown_ms'))"
done
bash tools/gpu_prof.sh ${T}_c4 python tools/bench_extra.py --workload c4 --steps 5 > gpurun_out/${T}_kstats.txt || exit 1
head -12 gpurun_out/${T}_kstats.txt
