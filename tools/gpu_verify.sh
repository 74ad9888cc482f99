# Round verification on one GPU: the full GPU suite, smoke, the default bench
# line (with its CPU baseline), rocprofv3 kernel stats of the C2 and C5 lines,
# and the supplementary workloads.  bash tools/gpu_verify.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-verify}
timeout -k 10 1000 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c2.jsonl 2>&1 || { tail -20 gpurun_out/${T}_bench_c2.jsonl; exit 1; }
tail -1 gpurun_out/${T}_bench_c2.jsonl | cut -c1-300
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/${T}_bench_c5.jsonl 2>&1 || { tail -20 gpurun_out/${T}_bench_c5.jsonl; exit 1; }
tail -1 gpurun_out/${T}_bench_c5.jsonl | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c2_stats -o run -- python bench.py --steps 5 --no-cpu-baseline > gpurun_out/${T}_c2_prof.txt 2>&1 || { tail -20 gpurun_out/${T}_c2_prof.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c5_stats -o run -- python bench.py --workload c5 --steps 5 --no-cpu-baseline > gpurun_out/${T}_c5_prof.txt 2>&1 || { tail -20 gpurun_out/${T}_c5_prof.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_sub_stats -o run -- python tools/bench_extra.py --workload subtract --steps 3 --warmup 1 > gpurun_out/${T}_sub_prof.txt 2>&1 || { tail -20 gpurun_out/${T}_sub_prof.txt; exit 1; }
for W in c3 c4 subtract window closest bed; do
  timeout -k 10 300 python tools/bench_extra.py --workload $W > gpurun_out/${T}_$W.jsonl 2>&1 || { tail -20 gpurun_out/${T}_$W.jsonl; exit 1; }
  echo "$W: $(grep '^{' gpurun_out/${T}_$W.jsonl | tail -1 | cut -c1-200)"
done
