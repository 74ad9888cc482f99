set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/rt_tests.txt 2>&1 || { tail -30 gpurun_out/rt_tests.txt; exit 1; }
tail -1 gpurun_out/rt_tests.txt
for lib in new build/rev_HEAD/liblime_amd.so; do
  unset LIME_AMD_LIB_VARIANT; [ "$lib" != new ] && export LIME_AMD_LIB_VARIANT=$PWD/$lib
  tag=rt_$(echo $lib | tr '/.' '__')
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python bench.py --sharded --no-ops --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/$tag.log 2>&1 || { tail -20 gpurun_out/$tag.log; exit 1; }
  echo "== $lib: $(grep '^{' gpurun_out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d['breakdown_ms'], d['config']['pairs_per_step'])")"
  python3 tools/kstats.py gpurun_out/$tag | grep -E "route|deinterleave"
done
