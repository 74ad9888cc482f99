set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-c5x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -k "bitset or c4 or c5 or contig_table or complement or genome_cut" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c5.txt 2>&1 || { tail -20 gpurun_out/${T}_c5.txt; exit 1; }
tail -1 gpurun_out/${T}_c5.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('breakdown_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o c5 -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof.txt 2>&1 || exit 1
python tools/rocpd_stats.py gpurun_out/${T}_prof/c5_results.db > gpurun_out/${T}_stats.csv && sed -n 1,10p gpurun_out/${T}_stats.csv
timeout -k 10 300 python tools/bench_extra.py --workload c4 > gpurun_out/${T}_c4.txt 2>&1 || { tail -20 gpurun_out/${T}_c4.txt; exit 1; }
tail -1 gpurun_out/${T}_c4.txt | cut -c1-700
