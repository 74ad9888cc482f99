# Round measurement: default bench line (with CPU baseline), kernel stats
# (rocprofv3 --kernel-trace --stats, CSV), and FETCH_SIZE / WRITE_SIZE PMC
# passes for the fill (separate runs; tools/pmc_summary.py applies the gfx950
# corrections).  Usage: bash tools/gpu_measure.sh TAG
set -e
tag=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run -- python bench.py --steps 5 --no-cpu-baseline > gpurun_out/${tag}_bench_prof.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${tag}_pmc_fetch.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${tag}_pmc_write.txt 2>&1
for w in c3 c4 c5 bed window closest; do
  timeout -k 10 300 python tools/bench_extra.py --workload $w > gpurun_out/${tag}_$w.txt 2>&1
done
