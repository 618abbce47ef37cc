#!/bin/bash
ROOT=$(pwd); OUT=$ROOT/gpurun_out/lmexp; mkdir -p $OUT; export TMPDIR=/tmp ITERS=3
cd /tmp
for v in lm_nomel; do
MIAUDIO_LIB=$ROOT/tools/probe/libmia_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace --kernel-include-regex fft_mel --output-format csv -d $OUT/$v -o run -- python3 $ROOT/tools/bench_logmel.py > $OUT/$v.log 2>&1 || exit $?
done
echo ok
