#!/bin/bash
# rocprofv3 kernel trace + stats of one bench configuration -> gpurun_out/prof_<tag>/trace
set -e
TAG=${1:-envnet}
ARGS=${2:-"--steps 5 --warmup 2 --no-cpu-baseline"}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $ROOT/bench.py $ARGS > $OUT/bench_trace.log 2>&1
echo done
