#!/bin/bash
# tools/probe/mg_variant.sh <name> "<-D flags>" -> tools/probe/libmia_<name>.so (mgemm.hip recompiled)
set -e
cd "$(dirname "$0")/../../dl-sound-classification_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable $2 -c csrc/mgemm.hip -o ../tools/probe/mgemm_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls build/*.o | grep -v build/mgemm.o) ../tools/probe/mgemm_$1.o -o ../tools/probe/libmia_$1.so
rm -f ../tools/probe/mgemm_$1.o ../tools/probe/libmia_$1.so.*
