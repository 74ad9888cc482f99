# Round-3 final verification, part 2: the supplementary workloads (C3, C4,
# subtract, window, closest, BED, the 1e9-row lines).  bash tools/gpu_verify3b.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-v3}
for W in c3 c4 subtract window closest bed b1_merge b1_pair; do
  timeout -k 10 300 python tools/bench_extra.py --workload $W > gpurun_out/${T}_$W.txt 2>&1 || { tail -20 gpurun_out/${T}_$W.txt; exit 1; }
  echo "$W: $(grep '^{' gpurun_out/${T}_$W.txt | tail -1 | cut -c1-250)"
done
