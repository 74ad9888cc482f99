# Round-end style verification on one GPU: full GPU suite, smoke, the default
# bench line, kernel stats, PMC bytes of the fill, the extra workloads.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r2v}
timeout -k 10 1000 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.txt 2>&1 || { tail -20 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt | cut -c1-400
for W in c3 c4 c5 subtract window closest bed; do
  if [ $W = c5 ]; then
    timeout -k 10 300 python bench.py --workload c5 > gpurun_out/${T}_$W.jsonl 2>&1 || { tail -20 gpurun_out/${T}_$W.jsonl; exit 1; }
  else
    timeout -k 10 300 python tools/bench_extra.py --workload $W > gpurun_out/${T}_$W.jsonl 2>&1 || { tail -20 gpurun_out/${T}_$W.jsonl; exit 1; }
  fi
  echo "$W: $(tail -1 gpurun_out/${T}_$W.jsonl | cut -c1-160)"
done
