# subtract with the count pass's per-row counts (default build) against the
# write pass folding every row twice (build/var_norc): subtract parity (scale
# tests included), then the sparse 1e9-row pairwise line and the C2-size
# subtract line, alternated
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-rc}
V=build/var_norc/liblime_amd.so
timeout -k 10 600 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_sharded.py -k "subtract" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
for L in "" $V "" $V; do
  timeout -k 10 300 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload subtract > gpurun_out/${T}_sub.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_sub.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('subtract var=${L:+norc}', round(d['ms_per_step'],3), d['breakdown_ms'])"
done
for L in "" $V; do
  timeout -k 10 400 env LIME_AMD_LIB_VARIANT=$L python tools/bench_extra.py --workload b1_pair --steps 1 > gpurun_out/${T}_b1.txt 2>&1 || exit 1
  grep -h '^{' gpurun_out/${T}_b1.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); b=d['breakdown_ms']; print('b1_pair var=${L:+norc}', round(d['ms_per_step'],2), {k: b[k] for k in ('subtract_lime_ms','subtract_set_ms','remnants_lime','remnants_set')})"
done
bash tools/gpu_prof.sh ${T}_b1 python tools/bench_extra.py --workload b1_pair --steps 1 > gpurun_out/${T}_kstats.txt || exit 1
head -12 gpurun_out/${T}_kstats.txt
