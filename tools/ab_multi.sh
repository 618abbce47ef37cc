#!/bin/bash
# Whole-step A/B over several builds of the C ABI (run through gpurun from the repo root):
#   bash tools/ab_multi.sh "<bench.py args>" name1 name2 ...   (name = tools/probe/libmia_<name>.so, or "base")
# alternating twice; one summary line per run, JSON lines in gpurun_out/abm/.
ARGS=$1; shift
OUT=gpurun_out/abm
mkdir -p $OUT
for i in 1 2; do
  for v in "$@"; do
    if [ $v = base ]; then LIBV=; else LIBV=$(realpath tools/probe/libmia_$v.so); fi
    MIAUDIO_LIB=$LIBV timeout -k 10 300 python -u bench.py $ARGS > $OUT/$v.$i.json 2> $OUT/$v.$i.err || exit 1
    python -c "import json,sys; d=json.loads(open('$OUT/$v.$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['ms_per_step'], {k: round(x['ms'], 3) for k, x in d.get('kernels', {}).items()})" | tee -a $OUT/summary.txt
  done
done
