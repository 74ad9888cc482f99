# Same-box A/B of whole source trees (their own Python + library): each
# tree's tools/bench_extra.py WORKLOAD, alternated ROUNDS times, then one
# rocprofv3 kernel-trace of each (kernel stats + the launch timeline).
#   XARGS="--steps 50" bash tools/ab_trees.sh TAG WORKLOAD ROUNDS tree1 tree2 ...   ("." = this tree)
# (trees from tools/build_rev.sh-style checkouts, e.g. build/tree_REV)
set -o pipefail
T=$1; W=$2; R=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
top=$PWD
for i in $(seq 1 $R); do for tr in "$@"; do
  tag=$(echo $tr | tr '/.' '__')
  out=$top/gpurun_out/${T}_${tag}_$i.txt
  (cd $tr && timeout -k 10 300 python tools/bench_extra.py --workload $W $XARGS > $out 2>&1) || { tail -20 $out; exit 1; }
  echo "$tr $i: $(grep '^{' $out | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), d.get('breakdown_ms'))")"
done; done
for tr in "$@"; do
  tag=$(echo $tr | tr '/.' '__')
  (cd $tr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $top/gpurun_out/${T}_${tag}_kt -o run -- python tools/bench_extra.py --workload $W $XARGS > $top/gpurun_out/${T}_${tag}_kt.log 2>&1) || { tail -20 $top/gpurun_out/${T}_${tag}_kt.log; exit 1; }
  python3 tools/kstats.py gpurun_out/${T}_${tag}_kt > gpurun_out/${T}_${tag}_kstats.txt
  echo "== $tr"; head -14 gpurun_out/${T}_${tag}_kstats.txt
done
