#!/bin/bash
# round-2 refresh: split-K weight gradients, GELU pass sizing, coalesced column sums, 4096 dGELU row walkers: full GPU suite, smoke, default bench line (both legs + CPU baselines), kernel
# traces + FETCH/WRITE PMC passes for both models
OUT=gpurun_out/r2t5; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo
bash tools/profile.sh envnet "--model envnet --steps 5 --warmup 2 --no-cpu-baseline" "--model envnet --steps 2 --warmup 1 --no-cpu-baseline" || exit $?
bash tools/profile.sh ast "--model ast --steps 3 --warmup 2 --no-cpu-baseline" "--model ast --steps 2 --warmup 1 --no-cpu-baseline" || exit $?
echo all-ok
