#!/bin/bash
# re-entry validation: full GPU suite + default bench line
OUT=gpurun_out/r2q; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/tests.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo
grep -o '"ast": {"metric[^,]*, "value": [0-9.]*' $OUT/bench.json
