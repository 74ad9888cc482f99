# the round's last changes on the default build: the new intersect parity
# tests, subtract, bitset extraction, smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-last}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "fill_windows or mixed_density or intersect_parity or subtract or bitset" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${T}_smoke.txt
