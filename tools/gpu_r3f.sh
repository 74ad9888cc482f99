# Round-3 f: per-wave split (bitset tests, C5 / C4 lines, C5 SQ counters),
# then the merge tile-geometry A/B on C3.  bash tools/gpu_r3f.sh TAG
set -o pipefail
T=${1:-r3f}
bash tools/gpu_c5.sh ${T} || exit $?
bash tools/gpu_ab.sh ${T}m "" "c3" new build/var_m256/liblime_amd.so
