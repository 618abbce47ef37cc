#!/bin/bash
# tools/probe/lm_variant.sh <name> "<-D flags>" -> tools/probe/libmia_<name>.so (logmel.hip recompiled)
set -e
cd "$(dirname "$0")/../../dl-sound-classification_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable $2 -c csrc/logmel.hip -o ../tools/probe/logmel_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls build/*.o | grep -v build/logmel.o) ../tools/probe/logmel_$1.o -o ../tools/probe/libmia_$1.so
rm -f ../tools/probe/logmel_$1.o ../tools/probe/libmia_$1.so.*
