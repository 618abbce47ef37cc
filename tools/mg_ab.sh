#!/bin/bash
# mgemm probe A/B (temporary): GEMM tests on the probe library, per-shape timing, AST step
V=$1
mkdir -p gpurun_out/mgab
MIAUDIO_LIB=$(realpath tools/probe/libmia_$V.so) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "mgemm or a_colsum" > gpurun_out/mgab/tests.log 2>&1 || { tail -30 gpurun_out/mgab/tests.log; exit 1; }
tail -1 gpurun_out/mgab/tests.log
SHAPES="qkv.fwd fc1.fwd fc2.fwd fc2.dgrad fc1.dgrad fc1.wgrad qkv.wgrad" bash tools/gemm_ab.sh $V > gpurun_out/mgab/gemm.txt 2>&1 || { tail -20 gpurun_out/mgab/gemm.txt; exit 1; }
grep -v amdgpu gpurun_out/mgab/gemm.txt | grep "path\|==" 
bash tools/ab_multi.sh "--model ast --steps 20 --warmup 5 --no-cpu-baseline" base $V
