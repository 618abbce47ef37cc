#!/bin/bash
# Staged GPU pass (through gpurun from the repo root).  STAGES picks the steps; each GPU step has its own
# limit and the chain stops at the first failure (a timeout / abort / fault ends the call).
#   STAGES="new bench attnpmc" NEW="tests/x.py" bash tools/gpu_stages.sh <tag>
TAG=${1:-r5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
( while sleep 45; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
export MIOPEN_FIND_MODE=FAST
STAGES=${STAGES:-"new tests smoke bench"}
NEW=${NEW:-""}
for s in $STAGES; do
  case $s in
    new)
      timeout -k 10 1000 python -u -m pytest $NEW -m gpu -v -s --timeout 600 --timeout-method thread > $OUT/new_tests.log 2>&1
      rc=$? ;;
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1
      rc=$? ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$? ;;
    bench)
      timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
      rc=$? ;;
    attnbwd)
      BATCH=${BATCH:-256} timeout -k 10 300 python -u tools/bench_attn_bwd.py > $OUT/attn_bwd.log 2>&1
      rc=$? ;;
    fc1upd)
      timeout -k 10 300 python -u tools/bench_fc1_update.py 256 512 1024 2048 > $OUT/fc1upd.log 2>&1
      rc=$? ;;
    stamps)
      BATCH=${BATCH:-256} timeout -k 10 200 python -u tools/attn_bwd_stamps.py > $OUT/stamps.log 2>&1
      rc=$? ;;
    attnpmc)
      bash tools/attn_bwd_pmc.sh $TAG/attnpmc > $OUT/attnpmc.log 2>&1
      rc=$? ;;
    *)
      echo "unknown stage $s"; exit 2 ;;
  esac
  echo "stage $s rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
