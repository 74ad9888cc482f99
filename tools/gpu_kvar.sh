# Kernel stats of one bench_extra workload per library variant (same box):
#   bash tools/gpu_kvar.sh TAG WORKLOAD "KERNEL_REGEX" lib1 lib2 ...   (lib "new" = in-tree)
set -o pipefail
T=$1; W=$2; K=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  unset LIME_AMD_LIB_VARIANT
  [ "$lib" != new ] && export LIME_AMD_LIB_VARIANT=$PWD/$lib
  tag=${T}_$(echo $lib | tr '/.' '__')
  timeout -k 10 ${KT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag} -o run -- python tools/bench_extra.py --workload $W > gpurun_out/${tag}.log 2>&1 || { tail -20 gpurun_out/${tag}.log; exit 1; }
  echo "== $lib: $(grep '^{' gpurun_out/${tag}.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('breakdown_ms'))")"
  python3 tools/kstats.py gpurun_out/${tag} | grep -E "$K"
done
