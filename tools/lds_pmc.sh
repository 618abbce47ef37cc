#!/bin/bash
# LDS bank-conflict pass (through gpurun from the repo root): SQ_LDS_BANK_CONFLICT against SQ_LDS_IDX_ACTIVE
# (the LDS-array cycles, MI355X_MICROARCH.md §LDS) per kernel, EnvNet and AST legs; summary: tools/lds_summary.py
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
for leg in envnet ast; do
  OUT=$ROOT/gpurun_out/lds_$leg
  mkdir -p $OUT
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv -d $OUT -o run -- python3 $ROOT/bench.py --model $leg --steps 2 --warmup 1 \
      --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
  echo "lds pass $leg ok"
done
