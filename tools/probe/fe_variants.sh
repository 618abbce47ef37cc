#!/bin/bash
# A/B builds of the product library with one source recompiled under experiment macros:
#   tools/probe/fe_variants.sh <src-stem> <name> "<-D flags>"   ->  tools/probe/libmia_<name>.so
# (the other objects are the product's build/*.o; run with MIAUDIO_LIB=tools/probe/libmia_<name>.so)
set -e
cd "$(dirname "$0")/../../dl-sound-classification_amd"
stem=$1; name=$2; flags=$3
extra=""
[ "$stem" = feconv ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
[ "$stem" = attention ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable \
  $extra $flags -c csrc/$stem.hip -o ../tools/probe/${stem}_$name.o
objs=$(ls build/*.o | grep -v "build/$stem.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs ../tools/probe/${stem}_$name.o -o ../tools/probe/libmia_$name.so
rm -f ../tools/probe/${stem}_$name.o ../tools/probe/libmia_$name.so.*
