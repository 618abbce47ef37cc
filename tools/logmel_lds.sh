#!/bin/bash
# log-mel LDS / VALU counters (through gpurun from the repo root): one pass over tools/bench_logmel.py
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/lmlds; mkdir -p $OUT
export TMPDIR=/tmp ITERS=3 ROUNDS=1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --kernel-include-regex "fft_mel" --output-format csv -d $OUT -o run -- python3 $ROOT/tools/bench_logmel.py > $OUT/run.log 2>&1 || exit $?
echo "lds pass ok"
