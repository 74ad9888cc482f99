# persistent double-buffered merge (build/var_m3q4, var_m3q8) against
# k_merge_scan2: merge parity under each variant, then C3 and C2 alternated
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-m3}
for L in build/var_m3q4/liblime_amd.so build/var_m3q8/liblime_amd.so; do
  timeout -k 10 400 env LIME_AMD_LIB_VARIANT=$L python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "merge or cluster or subtract or c3" > gpurun_out/${T}_tests.txt 2>&1
  rc=$?; echo "$L"; tail -2 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for L in "" build/var_m3q4/liblime_amd.so build/var_m3q8/liblime_amd.so; do
    timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload c3 > gpurun_out/${T}_c3.txt 2>&1 || exit 1
    grep -h '^{' gpurun_out/${T}_c3.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c3 var=$L', d['breakdown_ms'], round(d['roofline']['frac'],4))"
    timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python bench.py --steps 3 --no-cpu-baseline > gpurun_out/${T}_c2.txt 2>&1 || exit 1
    grep -h '^{' gpurun_out/${T}_c2.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c2 var=$L merge_ms', d['breakdown_ms']['merge_ms'])"
  done
done
