#!/bin/bash
# The driver's round-end GPU tiers in one call (through gpurun from the repo root): the whole -m gpu suite
# with -x as the driver runs it, smoke(), then the default bench line.  Each step has its own limit and the
# chain stops at the first failure.   bash tools/gpu_full.sh <tag> [bench args]
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export MIOPEN_FIND_MODE=FAST
( while sleep 45; do date +%T >> $OUT/hb.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1500 python -u -m pytest tests -x -m gpu -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py ${2:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -3 $OUT/gpu_tests.log
exit $rc
