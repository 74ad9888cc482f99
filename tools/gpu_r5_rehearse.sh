# Round-5 rehearsal of the driver's scaling command on a 1-GPU box: the
# default bench line at N = 2 over gloo (two ranks sharing the GPU, rows
# staged through the host), then the N = 1 line for comparison (pairs, runs,
# C3 runs / gaps and subtract records must be equal), then the C3 and 1e9
# merge-side lines as the sort baseline of this box.
#   bash tools/gpu_r5_rehearse.sh TAG
set -o pipefail
T=${1:-r5h}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_n1.log 2>&1 || { tail -30 gpurun_out/${T}_n1.log; exit 1; }
tail -c 2000 gpurun_out/${T}_n1.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 \
  --ops-steps 2 --dist-backend gloo > gpurun_out/${T}_n2_gloo.log 2>&1 || { tail -40 gpurun_out/${T}_n2_gloo.log; exit 1; }
grep '^{' gpurun_out/${T}_n2_gloo.log | tail -c 2000
for W in c3 b1_merge; do
  timeout -k 10 300 python tools/bench_extra.py --workload $W > gpurun_out/${T}_$W.log 2>&1 || { tail -20 gpurun_out/${T}_$W.log; exit 1; }
  grep '^{' gpurun_out/${T}_$W.log | tail -1
done
