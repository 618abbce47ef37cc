#!/bin/bash
# attention backward with / without the fused qkv bias sums: event timing + kernel trace
OUT=gpurun_out/r2z; mkdir -p $OUT
export BATCH=256 ITERS=5
timeout -k 10 120 python -u tools/bench_attn.py > $OUT/time.log 2>&1 || { cat $OUT/time.log; exit 1; }
cat $OUT/time.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
head -12 $(find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv" | head -1) | cut -c1-160
