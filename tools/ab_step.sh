#!/bin/bash
# Whole-step A/B on one GPU box (run through gpurun from the repo root):
#   bash tools/ab_step.sh "<bench.py args>" tools/probe/libmiaudio_ref.so
# runs bench.py with the product library, then with the given build of the same C ABI selected by
# MIAUDIO_LIB (src/miaudio/lib.py) -- the product .so is never touched -- alternating twice; JSON lines
# in gpurun_out/ab/.
ARGS=${1:-"--model ast --steps 5 --warmup 2 --no-cpu-baseline"}
REF=$2
OUT=gpurun_out/ab
mkdir -p $OUT
for i in 1 2; do
  for v in product ref; do
    if [ $v = ref ]; then LIBV=$(realpath $REF); else LIBV=; fi
    MIAUDIO_LIB=$LIBV timeout -k 10 300 python -u bench.py $ARGS > $OUT/$v.$i.json 2> $OUT/$v.$i.err || exit 1
    python -c "import json,sys; d=json.loads(open('$OUT/$v.$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['ms_per_step'], *[(k, d[k]['value']) for k in ('ast', 'ast_fp8') if k in d])"
  done
done
