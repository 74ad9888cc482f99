# sort stage check: sort tests, then kernel stats of the C2 bench (and C3)
set -o pipefail
mkdir -p gpurun_out
T=${1:-sc}
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sort.py > gpurun_out/${T}_sort.txt 2>&1 || { tail -30 gpurun_out/${T}_sort.txt; exit 1; }
tail -2 gpurun_out/${T}_sort.txt
bash tools/gpu_prof.sh ${T}_c2 python bench.py --steps 2 --warmup 1 --no-cpu-baseline | head -14
grep -h '^{' gpurun_out/${T}_c2_prof.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['breakdown_ms'])"
