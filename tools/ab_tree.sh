#!/bin/bash
# EnvNet step A/B: this tree vs an older tree checked out (and built) under tools/probe/<dir>
OUT=$(pwd)/gpurun_out/abtree; mkdir -p $OUT; OLD=tools/probe/$1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model envnet --steps 20 --warmup 5 --no-cpu-baseline > $OUT/new.$i.json 2> $OUT/new.$i.err || exit 1
  (cd $OLD && timeout -k 10 300 python -u bench.py --model envnet --steps 20 --warmup 5 --no-cpu-baseline > $OUT/old.$i.json 2> $OUT/old.$i.err) || exit 1
  for v in new old; do python -c "import json; d=json.loads(open('$OUT/$v.$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['ms_per_step'], {k: round(x['ms'], 3) for k, x in d.get('kernels', {}).items()})"; done
done
