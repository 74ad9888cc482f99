set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-so}
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c2.txt 2>&1 || { tail -20 gpurun_out/${T}_c2.txt; exit 1; }
tail -1 gpurun_out/${T}_c2.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown_ms'])"
timeout -k 10 300 python tools/bench_extra.py --workload c3 > gpurun_out/${T}_c3.txt 2>&1 || { tail -20 gpurun_out/${T}_c3.txt; exit 1; }
grep '^{' gpurun_out/${T}_c3.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['breakdown_ms'])"
