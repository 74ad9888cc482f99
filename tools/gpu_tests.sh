# Run GPU tests on the box: bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu "$@" > gpurun_out/${tag}_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.txt
exit $rc
