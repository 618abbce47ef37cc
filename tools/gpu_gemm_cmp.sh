#!/bin/bash
OUT=gpurun_out/gemmcmp; mkdir -p $OUT
TOKENS=421120 timeout -k 10 300 python -u tools/bench_gemm.py > $OUT/hand.log 2>&1 || { cat $OUT/hand.log; exit 1; }
TOKENS=421120 timeout -k 10 300 python -u tools/bench_gemm_lib.py > $OUT/lib.log 2>&1 || { cat $OUT/lib.log; exit 1; }
cat $OUT/hand.log $OUT/lib.log
