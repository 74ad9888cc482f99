set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r2l
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/${T}_c2.txt 2>&1 || { tail -20 gpurun_out/${T}_c2.txt; exit 1; }
tail -1 gpurun_out/${T}_c2.txt | cut -c1-1500
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/${T}_c5.txt 2>&1 || { tail -20 gpurun_out/${T}_c5.txt; exit 1; }
tail -1 gpurun_out/${T}_c5.txt | cut -c1-1500
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/${T}_c2_2r.txt 2>&1 || { tail -30 gpurun_out/${T}_c2_2r.txt; exit 1; }
grep metric gpurun_out/${T}_c2_2r.txt | cut -c1-1500
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --workload c5 --gpus 2 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/${T}_c5_2r.txt 2>&1 || { tail -30 gpurun_out/${T}_c5_2r.txt; exit 1; }
grep metric gpurun_out/${T}_c5_2r.txt | cut -c1-1500
