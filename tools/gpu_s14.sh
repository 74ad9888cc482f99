set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "intersect or scaled_c2 or stranded or subtract or full_size" > gpurun_out/s14_tests.txt 2>&1
timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/s14_bench.txt 2>&1
LIME_AMD_LIB_VARIANT=$PWD/build/var3/liblime_amd.so timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/s14_bench_var3.txt 2>&1
