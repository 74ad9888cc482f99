set -o pipefail
mkdir -p gpurun_out
T=${1:-r3f}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_sharded.py > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -le 1 ] || exit $rc
bash tools/gpu_prof.sh ${T}_c2 python bench.py --steps 3 --warmup 1 --no-cpu-baseline | head -14
grep -h '^{' gpurun_out/${T}_c2_prof.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], d['breakdown_ms'])"
