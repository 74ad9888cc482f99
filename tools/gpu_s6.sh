set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s6_prof -o run -- python bench.py --steps 5 --no-cpu-baseline > gpurun_out/s6_bench.txt 2>&1
