# Quick GPU check after a kernel change: named tests, then a bench line with
# rocprofv3 kernel stats.  bash tools/gpu_quick.sh TAG "pytest args" "bench cmd"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; TESTS=$2; BENCH=$3
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread $TESTS > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_stats -o run -- python $BENCH > gpurun_out/${T}_bench.txt 2>&1
rc=$?; grep '^{' gpurun_out/${T}_bench.txt | cut -c1-200; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.txt; exit $rc; }
grep -h '^{' gpurun_out/${T}_bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d.get('breakdown_ms'), d.get('ms_per_step'))"
python3 tools/kstats.py gpurun_out/${T}_stats | head -24
