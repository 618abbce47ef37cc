#!/bin/bash
# log-mel timing + SQ counter passes (tools/bench_logmel.py), from the repo root via gpurun
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-logmel}
mkdir -p $OUT
export TMPDIR=/tmp ITERS=${ITERS:-3}
timeout -k 10 120 python3 -u $ROOT/tools/bench_logmel.py > $OUT/time.log 2>&1 || { cat $OUT/time.log; exit 1; }
cat $OUT/time.log
cd /tmp
RX='fft_mel|clip_'
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $OUT/a -o run -- python3 $ROOT/tools/bench_logmel.py > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $OUT/b -o run -- python3 $ROOT/tools/bench_logmel.py > $OUT/b.log 2>&1 || exit $?
echo "logmel pmc ok"
cd $ROOT && timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_logmel.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
