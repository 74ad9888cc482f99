# Whole-library variant built from a git revision, for same-box A/B against
# an earlier commit (tools/gpu_ab.sh build/rev_REV/liblime_amd.so):
#   bash tools/build_rev.sh REV   -> build/rev_REV/liblime_amd.so
set -e
rev=$1
d=build/rev_$rev
rm -rf "$d"
mkdir -p "$d/src"
git archive "$rev" lime_amd/csrc include | tar -x -C "$d/src"
make -j8 LIB="$d/liblime_amd.so" OBJDIR="$d/obj" SRC="$d/src/lime_amd/csrc" "$d/liblime_amd.so" > "$d/build.log" 2>&1 || { tail -20 "$d/build.log"; exit 1; }
rm -rf "$d/obj" "$d/src"
echo "$d/liblime_amd.so"
