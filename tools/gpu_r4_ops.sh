# Round-4: the new bench workloads.  1 GPU: c2 with its operators lines (c3
# merge side, subtract), then c3 and sub on their own; 2 ranks sharing the GPU
# over gloo (rehearsal of the sharded paths): c3, sub, c2 with operators.
#   bash tools/gpu_r4_ops.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4o}
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c2ops_1.txt 2>&1 || { tail -30 gpurun_out/${T}_c2ops_1.txt; exit 1; }
grep '^{' gpurun_out/${T}_c2ops_1.txt | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step']); [print(k, v['value'], v['ms_per_step'], {x: v[x] for x in v if x in ('runs','gaps','records')}) for k, v in d['operators'].items()]"
for W in c3 sub; do
  timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 1 > gpurun_out/${T}_${W}_1.txt 2>&1 || { tail -30 gpurun_out/${T}_${W}_1.txt; exit 1; }
  grep '^{' gpurun_out/${T}_${W}_1.txt | tail -1 | cut -c1-500
done
for W in c3 sub c2; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --workload $W --dist-backend gloo --no-cpu-baseline --ops-steps 1 > gpurun_out/${T}_${W}_2r.txt 2>&1 || { tail -30 gpurun_out/${T}_${W}_2r.txt; exit 1; }
  grep '^{' gpurun_out/${T}_${W}_2r.txt | tail -1 | cut -c1-700
done
