set -e
mkdir -p gpurun_out
for lib in default var2; do for g in 2048 1000000; do for sp in 131072 0; do
  if [ $lib = var2 ]; then export LIME_AMD_LIB_VARIANT=$PWD/build/var2/liblime_amd.so; else unset LIME_AMD_LIB_VARIANT; fi
  LIME_FILL_GRAN=$g LIME_FILL_SPAN=$sp timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/s13_${lib}_${g}_$sp.txt 2>&1
done; done; done
