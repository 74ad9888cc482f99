set -o pipefail
mkdir -p gpurun_out
T=${1:-r3e}
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --ignore tests/test_gpu_scale.py > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -12 gpurun_out/${T}_tests.txt; [ $rc -le 1 ] || exit $rc
bash tools/gpu_ab.sh ${T}ab "" "c2" new build/var_blk/liblime_amd.so
