# One parameterised GPU driver (replaces the per-round gpu_r4_* / gpu_r5_* /
# gpu_verify* scripts).  Each step runs under its own time limit, writes
# gpurun_out/TAG_<step>.txt and stops the script on any failure.
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
# steps:
#   suite | suite:KEXPR   pytest -m gpu (optionally -k KEXPR)
#   smoke                 __graft_entry__.smoke()
#   bench:W               bench.py --workload W (the full line, CPU baseline included)
#   rehearse:N            bench.py --gpus N --dist-backend gloo (its own N ranks sharing one GPU)
#   prof:W                rocprofv3 --kernel-trace --stats of bench.py --workload W (c2 c5 c3 sub)
#                         or of tools/bench_extra.py --workload W (anything else)
#   extra:W               tools/bench_extra.py --workload W
#   pmc:W                 FETCH_SIZE and WRITE_SIZE passes (one --pmc run each) + per-kernel bytes
#   sq:W                  SQ issue / stall / LDS counters, one --pmc pass
#   pmcjson:SHA           profiles/pmc_c2.json / pmc_c5.json inputs for bench.py's "traffic"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; shift
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${T}_${name}.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/${T}_${name}.txt | cut -c1-600
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/${T}_${name}.txt; exit $rc; fi
}
prog() {  # workload -> the python program + args that run it briefly
  case $1 in
    c2) echo "bench.py --steps 5 --warmup 2 --no-cpu-baseline" ;;
    c5|c3|sub) echo "bench.py --workload $1 --steps 5 --warmup 2 --no-cpu-baseline" ;;
    *) echo "tools/bench_extra.py --workload $1" ;;
  esac
}
SQC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS"
for S in "$@"; do
  k=${S%%:*}; a=${S#*:}; [ "$a" = "$S" ] && a=
  case $k in
    suite)
      if [ -n "$a" ]; then
        run suite 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests -k "$a"
      else
        run suite 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests
      fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_$a 500 python bench.py --workload $a ;;
    rehearse) run rehearse_$a 1000 python bench.py --gpus $a --dist-backend gloo --steps 2 \
                --warmup 1 --ops-steps 2 ;;
    prof)
      run prof_$a 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/${T}_${a}_stats -o run -- python $(prog $a)
      python3 tools/kstats.py gpurun_out/${T}_${a}_stats > gpurun_out/${T}_${a}_kstats.txt; head -16 gpurun_out/${T}_${a}_kstats.txt ;;
    extra) run extra_$a 300 python tools/bench_extra.py --workload $a ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_${a}_$C \
          -o p -- python $(prog $a) > gpurun_out/${T}_${a}_$C.log 2>&1 \
          || { tail -5 gpurun_out/${T}_${a}_$C.log; exit 1; }
      done
      python3 tools/pmc_summary.py gpurun_out/${T}_${a}_FETCH_SIZE gpurun_out/${T}_${a}_WRITE_SIZE \
        > gpurun_out/${T}_${a}_bytes.txt && head -40 gpurun_out/${T}_${a}_bytes.txt ;;
    sq)
      timeout -s KILL 300 rocprofv3 --pmc $SQC --output-format csv -d gpurun_out/${T}_${a}_sq \
        -o p -- python $(prog $a) > gpurun_out/${T}_${a}_sq.log 2>&1 \
        || { tail -5 gpurun_out/${T}_${a}_sq.log; exit 1; }
      python3 tools/pmc_summary.py gpurun_out/${T}_${a}_sq > gpurun_out/${T}_${a}_sq_summary.txt
      head -60 gpurun_out/${T}_${a}_sq_summary.txt ;;
    pmcjson)
      c2="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops"
      c5="python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline"
      for W in c2 c5; do
        cmd=${!W}
        for C in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${T}_${W}_$C \
            -o p -- $cmd > gpurun_out/${T}_${W}_$C.log 2>&1 \
            || { tail -5 gpurun_out/${T}_${W}_$C.log; exit 1; }
        done
      done
      python3 tools/pmc_json.py gpurun_out/${T}_pmc_c2.json gpurun_out/${T}_c2_FETCH_SIZE \
        gpurun_out/${T}_c2_WRITE_SIZE --commit "$a" --cmd "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- $c2" \
        --key "k_fill<1, false, false>" || exit 1
      python3 tools/pmc_json.py gpurun_out/${T}_pmc_c5.json gpurun_out/${T}_c5_FETCH_SIZE \
        gpurun_out/${T}_c5_WRITE_SIZE --commit "$a" --cmd "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- $c5" \
        --steps 3 --exclude k_uniform || exit 1 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
