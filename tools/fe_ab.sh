#!/bin/bash
# frontend kernel A/B: tools/bench_fe.py on the product library and tools/probe/libmia_<name>.so builds
OUT=gpurun_out/${TAG:-feab}; mkdir -p $OUT
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then LIBV=; else LIBV=$(realpath tools/probe/libmia_$v.so); fi
    echo "== $v $i" >> $OUT/ab.log
    MIAUDIO_LIB=$LIBV timeout -k 10 120 python -u tools/bench_fe.py ${KERNELS:-fe_conv3_fwd fe_conv1_fwd} >> $OUT/ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu $OUT/ab.log
