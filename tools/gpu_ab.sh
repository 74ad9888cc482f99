# A/B of library variants on one box: GPU tests (-k EXPR) on the new library,
# then each workload's bench line per variant.
#   [XARGS="--steps 50"] bash tools/gpu_ab.sh TAG "pytest -k expr" "c2 c3 ..." lib1 lib2 ...
# (lib "new" = lime_amd/liblime_amd.so; c2 / c5 via bench.py, others bench_extra)
set -o pipefail
tag=$1; kexpr=$2; works=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests -k "$kexpr" > gpurun_out/${tag}_tests.txt 2>&1 || { tail -40 gpurun_out/${tag}_tests.txt; exit 1; }
  tail -1 gpurun_out/${tag}_tests.txt
fi
for i in $(seq 1 ${ROUNDS:-2}); do for lib in "$@"; do for W in $works; do
  # "new:VAR=VAL" = the new library with one environment setting
  unset LIME_AMD_LIB_VARIANT
  case $lib in
    new) ;;
    new:*) ev=${lib#new:}; export "$ev" ;;
    *) export LIME_AMD_LIB_VARIANT=$PWD/$lib ;;
  esac
  out=gpurun_out/${tag}_$(echo $lib | tr '/:=' '___')_${W}_$i.txt
  case $W in
    c2) timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ops > $out 2>&1 ;;
    c5) timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $out 2>&1 ;;
    *) timeout -k 10 300 python tools/bench_extra.py --workload $W $XARGS > $out 2>&1 ;;
  esac || { tail -20 $out; exit 1; }
  echo "$lib $W $i: $(grep '^{' $out | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('breakdown_ms'))")"
  if [ "${lib#new:}" != "$lib" ]; then unset "${ev%%=*}"; fi
done; done; done
