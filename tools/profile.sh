#!/bin/bash
# GPU-box profiling recipe (run through gpurun from the repo root):
#   rocprofv3 kernel-trace + stats of the bench, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, and
#   'sq': MFMA-busy / wait / LDS counters, 8 SQ counters in one pass),
#   each pass its own run with only --kernel-trace beside --pmc (no sys/runtime trace with counters).
# Outputs under gpurun_out/prof_<tag>/ ; tools/pmc_summary.py condenses them into profiles/.
set -e
TAG=${1:-envnet}
ARGS=${2:-"--steps 5 --warmup 2 --no-cpu-baseline"}
PMC_ARGS=${3:-"--steps 2 --warmup 1 --no-cpu-baseline"}
PASSES=${4:-"trace fetch write"}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for p in $PASSES; do
  case $p in
    trace) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
             python3 $ROOT/bench.py $ARGS > $OUT/bench_trace.log 2>&1 ;;
    fetch) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
             python3 $ROOT/bench.py $PMC_ARGS > $OUT/bench_fetch.log 2>&1 ;;
    write) timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
             python3 $ROOT/bench.py $PMC_ARGS > $OUT/bench_write.log 2>&1 ;;
    sq)    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
             SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace \
             --output-format csv -d $OUT/sq -o run -- python3 $ROOT/bench.py $PMC_ARGS > $OUT/bench_sq.log 2>&1 ;;
  esac
  echo "pass $p ok"
done
