#!/bin/bash
# log-mel: parity tests + timing + SQ counters
OUT=gpurun_out/r2z; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_logmel.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -30; exit $rc; }
bash tools/logmel_pmc.sh r2z_pmc
