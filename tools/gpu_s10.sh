set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/fill_exp.py > gpurun_out/s10_fill.txt 2>&1
LIME_FILL_DRY=1 timeout -k 10 200 python tools/fill_exp.py > gpurun_out/s10_dry.txt 2>&1
