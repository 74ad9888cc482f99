set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-t}; shift
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu "$@" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
