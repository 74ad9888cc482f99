set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-cl}
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_closest.py tests/test_cli.py tests/test_gpu_parity.py -k "closest or genome_cut" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_p -o s -- python tools/bench_extra.py --workload closest > gpurun_out/${T}.jsonl 2>&1 || { tail -5 gpurun_out/${T}.jsonl; exit 1; }
grep '^{' gpurun_out/${T}.jsonl | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown_ms'])"
python tools/rocpd_stats.py gpurun_out/${T}_p/s_results.db > gpurun_out/${T}_stats.csv && sed -n 1,16p gpurun_out/${T}_stats.csv
