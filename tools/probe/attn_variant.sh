#!/bin/bash
# tools/probe/attn_variant.sh <name> "<-D flags>" -> tools/probe/libmia_<name>.so (attention.hip recompiled
# with the Makefile's flags for it)
set -e
cd "$(dirname "$0")/../../dl-sound-classification_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize $2 -c csrc/attention.hip -o ../tools/probe/attention_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls build/*.o | grep -v build/attention.o) ../tools/probe/attention_$1.o -o ../tools/probe/libmia_$1.so
rm -f ../tools/probe/attention_$1.o ../tools/probe/libmia_$1.so.*
