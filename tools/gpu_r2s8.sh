#!/bin/bash
# two-rank gradient exchange with the real HIP backward (gloo on one GPU)
OUT=gpurun_out/r2s8; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_ddp.py -x -v --timeout 650 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
exit $rc
