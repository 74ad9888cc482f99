# rocprofv3 kernel stats of one command: bash tools/gpu_prof.sh TAG cmd...
# -> gpurun_out/TAG_stats/ (csv) and a short per-kernel summary on stdout
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_stats -o run -- "$@" > gpurun_out/${T}_prof.txt 2>&1 || { tail -20 gpurun_out/${T}_prof.txt; exit 1; }
python3 tools/kstats.py gpurun_out/${T}_stats
