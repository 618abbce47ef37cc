#!/bin/bash
# GPU-box driver for one gpurun call: pytest selection, then (unless pytest crashed) the bench.
#   bash tools/gpu_run.sh "<pytest args>" "<bench args or 'skip'>" [tag]
ROOT=$(pwd)
TAG=${3:-run}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
rc=0
if [ "$1" != "skip" ]; then
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread $1 > $OUT/tests.log 2>&1
  rc=$?
  tail -5 $OUT/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ "$2" != "skip" ]; then
  timeout -k 10 600 python -u bench.py $2 > $OUT/bench.json 2> $OUT/bench.err
  brc=$?
  echo "bench rc=$brc"; tail -c 3000 $OUT/bench.json
  [ $brc -ne 0 ] && tail -20 $OUT/bench.err && exit $brc
fi
exit $rc
