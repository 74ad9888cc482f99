set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s30_tests.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s30_smoke.txt 2>&1
timeout -k 10 300 python bench.py > gpurun_out/s30_bench.txt 2>&1
