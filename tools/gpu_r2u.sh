#!/bin/bash
# round-2 validation: full GPU suite, default bench, kernel traces + HBM PMC passes for both models
OUT=gpurun_out/r2u; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/tests.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 600 $OUT/bench.json; echo
bash tools/profile.sh envnet "--model envnet --steps 5 --warmup 2 --no-cpu-baseline" "--model envnet --steps 2 --warmup 1 --no-cpu-baseline" || exit $?
bash tools/profile.sh ast "--model ast --steps 3 --warmup 2 --no-cpu-baseline" "--model ast --steps 2 --warmup 1 --no-cpu-baseline" || exit $?
echo all-ok
