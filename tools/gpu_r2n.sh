#!/bin/bash
OUT=gpurun_out/r2n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm.py -k "bgrad or plain" > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" $OUT/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
TOKENS=421120 timeout -k 10 300 python -u tools/bench_gemm.py > $OUT/gemm.log 2>&1 || { tail $OUT/gemm.log; exit 1; }
grep -E "wgrad" $OUT/gemm.log
