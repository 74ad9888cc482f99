set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r2u}
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_threads.py tests/test_gpu_sharded.py > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c2.txt 2>&1 || { tail -20 gpurun_out/${T}_c2.txt; exit 1; }
tail -1 gpurun_out/${T}_c2.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown_ms'], d['roofline']['avg_launch_ms'])"
