set -e
mkdir -p gpurun_out
timeout -k 10 200 ./bin/alloc_probe > gpurun_out/s24_alloc.jsonl 2>&1
timeout -k 10 200 ./bin/alloc_probe > gpurun_out/s24_alloc2.jsonl 2>&1
