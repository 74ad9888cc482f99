# 2-rank rehearsal of the sharded bench on one GPU (gloo: RCCL cannot put two ranks on one device)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r2x}
for W in c2 c5; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --workload $W --dist-backend gloo --no-cpu-baseline > gpurun_out/${T}_$W.txt 2>&1 || { tail -30 gpurun_out/${T}_$W.txt; exit 1; }
  grep '^{' gpurun_out/${T}_$W.txt | tail -1 | cut -c1-400
done
