#!/bin/bash
# clip + Adam tensor-order A/B on one box
OUT=gpurun_out/r2s11; mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_adam.py > $OUT/adam.log 2>&1; rc=$?
cat $OUT/adam.log | tail -3
exit $rc
