#!/bin/bash
# Profiling pass (through gpurun from the repo root): default bench line, then for each leg the
# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE / SQ passes (tools/profile.sh), each step under its
# own time limit; outputs in gpurun_out/prof_<leg>/ and gpurun_out/$PTAG/.
OUT=gpurun_out/${PTAG:-r5prof}
mkdir -p $OUT
( while sleep 45; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
LEGS=${LEGS:-"envnet ast ast-fp8"}
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
fi
for leg in $LEGS; do
  bash tools/profile.sh $leg "--model $leg --steps 3 --warmup 2 --no-cpu-baseline" \
      "--model $leg --steps 2 --warmup 1 --no-cpu-baseline" "trace fetch write sq" > $OUT/prof_$leg.log 2>&1 || exit $?
done
echo "profile ok"
