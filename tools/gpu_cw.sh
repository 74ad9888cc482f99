# subtract count-pass workgroup size: 4 waves (default) against 2 and 8
# (build/var_cw2, var_cw8): subtract parity per variant, then the C2-size
# subtract and the sparse 1e9-row pairwise line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-cw}
for L in build/var_cw2/liblime_amd.so build/var_cw8/liblime_amd.so; do
  timeout -k 10 400 env LIME_AMD_LIB_VARIANT=$L python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "subtract" > gpurun_out/${T}_tests.txt 2>&1
  rc=$?; echo "$L"; tail -1 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
done
for L in "" build/var_cw2/liblime_amd.so build/var_cw8/liblime_amd.so; do
  timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload subtract > gpurun_out/${T}_sub.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_sub.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('subtract var=$L', round(d['ms_per_step'],3), d['breakdown_ms'])"
  timeout -k 10 400 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload b1_pair --steps 1 > gpurun_out/${T}_b1.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_b1.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); b=d['breakdown_ms']; print('b1_pair var=$L', round(d['ms_per_step'],2), {k: b[k] for k in ('subtract_lime_ms','subtract_set_ms')})"
done
