# Round-4 combined check: GPU tests (KEXPR), the same tests on a variant
# library (VLIB / VEXPR), then bench A/B lines (ABW over LIBS) and the
# bench workloads' operators lines (tools/gpu_r4_ops.sh).
#   KEXPR=... VLIB=... VEXPR=... ABW=... LIBS=... PROF=... bash tools/gpu_r4_round.sh TAG
# (PROF: bench_extra workloads profiled with kernel stats)
set -o pipefail
T=${1:-r4r}
if [ -n "$KEXPR" ]; then KEXPR="$KEXPR" WORKS="$PROF" bash tools/gpu_r4_check.sh ${T}k || exit 1; fi
if [ -n "$VLIB" ]; then LIME_AMD_LIB_VARIANT=$PWD/$VLIB KEXPR="$VEXPR" WORKS= bash tools/gpu_r4_check.sh ${T}v || exit 1; fi
if [ -n "$ABW" ]; then bash tools/gpu_ab.sh ${T}ab "" "$ABW" $LIBS || exit 1; fi
if [ -n "$OPS" ]; then bash tools/gpu_r4_ops.sh ${T}o || exit 1; fi
