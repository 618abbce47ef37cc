#!/bin/bash
# attention-only GPU iteration: parity tests, timing at B=256, SQ counters at B=64
OUT=gpurun_out/${1:-attn_it}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_ast.py -k attention > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -gt 1 ] && exit $rc
BATCH=256 timeout -k 10 300 python -u tools/bench_attn.py > $OUT/attn.log 2>&1 || exit $?
cat $OUT/attn.log
BATCH=64 bash tools/attn_pmc.sh ${1:-attn_it}/pmc || exit $?
python tools/sq_summary.py $OUT/pmc
