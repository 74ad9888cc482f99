# Whole-library variant of the in-tree sources built with extra defines, for
# same-box A/B of one kernel's compile-time knobs (tools/gpu_kvar.sh):
#   bash tools/build_var.sh NAME "-DLIME_X=1 -DLIME_Y=2"  -> build/var_NAME/liblime_amd.so
set -e
name=$1; defs=$2
d=build/var_$name
rm -rf "$d"; mkdir -p "$d"
HF="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-variable -Wno-unused-result $defs"
make -j8 LIB="$d/liblime_amd.so" OBJDIR="$d/obj" HIPFLAGS="$HF" "$d/liblime_amd.so" > "$d/build.log" 2>&1 || { tail -20 "$d/build.log"; exit 1; }
rm -rf "$d/obj"
echo "$d/liblime_amd.so"
