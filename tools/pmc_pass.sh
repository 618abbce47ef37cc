#!/bin/bash
# One rocprofv3 PMC pass (counters only beside --kernel-trace) over a short bench run.
#   bash tools/pmc_pass.sh <tag> "<counters>" "<bench args>" [kernel-regex]
set -e
TAG=$1; CTR=$2; ARGS=${3:-"--steps 2 --warmup 1 --no-cpu-baseline"}; RX=${4:-""}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
EXTRA=()
if [ -n "$RX" ]; then EXTRA=(--kernel-include-regex "$RX"); fi
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace "${EXTRA[@]}" --output-format csv -d $OUT -o run -- \
    python3 $ROOT/bench.py $ARGS > $OUT/bench.log 2>&1
echo "pmc $TAG ok"
