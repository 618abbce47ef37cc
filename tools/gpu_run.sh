#!/bin/bash
# The one GPU-box recipe of this repo (run through gpurun from the repo root):
#   bash tools/gpu_run.sh TAG "<pytest args | skip>" "<bench.py args | skip>" ["<extra command | skip>"]
# 1. pytest with the given args (thread-method timeout per test), log in gpurun_out/TAG/tests.log;
#    an assertion failure (rc 1) still lets the bench run, anything worse (crash, abort, timeout) stops;
# 2. bench.py with the given args, JSON line in gpurun_out/TAG/bench.json, progress in bench.err;
# 3. an optional extra command (a profile pass, a micro-bench), output in gpurun_out/TAG/extra.log.
# Every GPU step runs under its own `timeout -k 10`.
ROOT=$(pwd)
TAG=${1:-run}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
rc=0
if [ "${2:-skip}" != "skip" ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread $2 > "$OUT/tests.log" 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|^\[" "$OUT/tests.log" | tail -40
  tail -3 "$OUT/tests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ "${3:-skip}" != "skip" ]; then
  timeout -k 10 600 python -u bench.py $3 > "$OUT/bench.json" 2> "$OUT/bench.err"
  brc=$?
  echo "bench rc=$brc"; tail -c 2500 "$OUT/bench.json"
  if [ $brc -ne 0 ]; then tail -20 "$OUT/bench.err"; exit $brc; fi
fi
if [ "${4:-skip}" != "skip" ]; then
  timeout -k 10 600 bash -c "$4" > "$OUT/extra.log" 2>&1
  erc=$?
  echo "extra rc=$erc"; tail -30 "$OUT/extra.log"
  [ $erc -ne 0 ] && exit $erc
fi
exit $rc
