# Rehearsal of the driver's scaling command at N = 4 on a 1-GPU box: four
# ranks over gloo sharing the GPU (rows staged through the host).  Pairs, runs,
# C3 runs / gaps and subtract records must equal the N = 1 line's.
#   bash tools/gpu_r5_rehearse4.sh TAG
set -o pipefail
T=${1:-r5h4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 2 --warmup 1 \
  --ops-steps 2 --dist-backend gloo > gpurun_out/${T}_n4_gloo.log 2>&1 || { tail -40 gpurun_out/${T}_n4_gloo.log; exit 1; }
grep '^{' gpurun_out/${T}_n4_gloo.log | tail -c 3000
