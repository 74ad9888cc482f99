# A/B timing of library variants on one box: tools/ab.sh TAG lib1 lib2 ...
# (paths relative to the repo; "new" = lime_amd/liblime_amd.so)
set -e
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do for lib in "$@"; do
  if [ "$lib" = new ]; then unset LIME_AMD_LIB_VARIANT; else export LIME_AMD_LIB_VARIANT=$PWD/$lib; fi
  name=$(echo $lib | tr '/' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_${name}_$i -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_${name}_$i.txt 2>&1
done; done
