#!/bin/bash
# Epilogue ablations of the AST GEMM shapes (tools/bench_gemm.py name:epilogue) on the product library and
# on tools/probe/libmia_<name>.so builds given as arguments.
OUT=gpurun_out/${TAG:-gemmepi}; mkdir -p $OUT
SHAPES=${SHAPES:-"fc1.fwd:gelu_save_d fc1.fwd:gelu fc1.fwd:plain fc2.dgrad:dmul fc2.dgrad:dmul_nocs fc2.dgrad:plain proj.fwd:residual proj.fwd:f32 proj.fwd:plain fc2.fwd:residual fc2.fwd:f32"}
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then LIBV=; else LIBV=$(realpath tools/probe/libmia_$v.so); fi
    echo "== $v $i" >> $OUT/ab.log
    MIAUDIO_LIB=$LIBV REPS=10 timeout -k 10 200 python -u tools/bench_gemm.py $SHAPES >> $OUT/ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu $OUT/ab.log
