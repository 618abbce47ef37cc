#!/bin/bash
# mgemm A/B: tools/bench_gemm.py on the product library and on tools/probe/libmia_<name>.so builds,
# interleaved twice; CHECKSUM=1 adds a sha1 of each shape's outputs (bit-for-bit comparison across builds).
#   SHAPES="fc1.fwd qkv.fwd" bash tools/gemm_ab.sh <tag> name1 name2 ...
TAG=${1:-gemmab}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
SHAPES=${SHAPES:-"qkv.fwd fc1.fwd fc2.dgrad fc1.dgrad qkv.dgrad"}
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then LIBV=; else LIBV=$(realpath tools/probe/libmia_$v.so); fi
    echo "== $v $i" >> $OUT/ab.log
    MIAUDIO_LIB=$LIBV REPS=10 timeout -k 10 200 python -u tools/bench_gemm.py $SHAPES >> $OUT/ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu $OUT/ab.log
