# Kernel stats of one workload under two settings of one variable:
#   bash tools/gpu_kstats_env.sh TAG WORKLOAD VAR=VAL
# (WORKLOAD c2 / c5: bench.py; others: tools/bench_extra.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; W=$2; EV=$3
case $W in
  c2|c5) P="bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline" ;;
  *) P="tools/bench_extra.py --workload $W --steps 3 --warmup 1" ;;
esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_a -o run -- python $P > gpurun_out/${T}_a.log 2>&1 || { tail -5 gpurun_out/${T}_a.log; exit 1; }
export "$EV"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_b -o run -- python $P > gpurun_out/${T}_b.log 2>&1 || { tail -5 gpurun_out/${T}_b.log; exit 1; }
for x in a b; do
  echo "== $x"
  python - gpurun_out/${T}_$x/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.reader(open(sys.argv[1])))[1:14]
for r in rows:
    n = r[0].split("(anonymous namespace)::")[-1][:48]
    print(f"  {n:50s} calls={r[1]:>4s} avg_us={float(r[3]) / 1000:9.1f}")
PY
done
