# thread-per-owner fill for sparse plans (build/var_sparse) against k_fill
# everywhere (the default build): intersect / window / closest parity under
# the variant (the 1e9-row intersect included), then the sparse 1e9-row line
# and window, alternated
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-sp}
V=build/var_sparse/liblime_amd.so
timeout -k 10 700 env LIME_AMD_LIB_VARIANT=$V python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py tests/test_closest.py tests/test_gpu_threads.py tests/test_gpu_streams.py tests/test_gpu_scale.py -k "intersect or window or closest or pair or c2 or thread or stream or fill" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for L in $V "" $V ""; do
  timeout -k 10 400 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload b1_pair --steps 1 > gpurun_out/${T}_b1.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_b1.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); b=d['breakdown_ms']; print('b1_pair var=${L:+sparse}', round(d['ms_per_step'],2), {k: b[k] for k in ('count_ms','fill_ms','pairs')})"
done
LIME_AMD_LIB_VARIANT=$V bash tools/gpu_prof.sh ${T}_b1 python tools/bench_extra.py --workload b1_pair --steps 1 > gpurun_out/${T}_kstats.txt || exit 1
head -8 gpurun_out/${T}_kstats.txt
