set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r2t
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -k "bitset or c4 or c5 or ops or contig_table or merge or intersect" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c5.txt 2>&1 || { tail -20 gpurun_out/${T}_c5.txt; exit 1; }
tail -1 gpurun_out/${T}_c5.txt | cut -c1-900
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c2.txt 2>&1 || { tail -20 gpurun_out/${T}_c2.txt; exit 1; }
tail -1 gpurun_out/${T}_c2.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown_ms'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o c5 -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof.txt 2>&1 || exit 1
f=$(ls gpurun_out/${T}_prof/*/c5_kernel_stats.csv | tail -1); cut -d, -f1-5 $f | head -14
