#!/bin/bash
# attention backward A/B: product library vs tools/probe/libmia_<name>.so (bench_attn_bwd.py), then the
# attention parity tests on the product library
OUT=gpurun_out/attnab; mkdir -p $OUT
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then LIBV=; else LIBV=$(realpath tools/probe/libmia_$v.so); fi
    echo "== $v $i" >> $OUT/ab.log
    MIAUDIO_LIB=$LIBV BATCH=256 ROUNDS=2 timeout -k 10 200 python -u tools/bench_attn_bwd.py >> $OUT/ab.log 2>&1 || exit 1
  done
done

