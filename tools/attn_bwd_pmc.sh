#!/bin/bash
# SQ counter passes over tools/bench_attn_bwd.py (fused vs two-kernel backward; run through gpurun from the
# repo root):  bash tools/attn_bwd_pmc.sh <tag>   -> gpurun_out/<tag>/{a,b}; python tools/sq_summary.py
ROOT=$(pwd)
TAG=${1:-attnbwd}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp BATCH=${BATCH:-64} ITERS=${ITERS:-2} ROUNDS=1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --kernel-include-regex attn --output-format csv -d $OUT/a -o run -- python3 $ROOT/tools/bench_attn_bwd.py > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace --kernel-include-regex attn --output-format csv -d $OUT/b -o run -- python3 $ROOT/tools/bench_attn_bwd.py > $OUT/b.log 2>&1 || exit $?
echo "attn bwd pmc ok"
