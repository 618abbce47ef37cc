#!/bin/bash
# mg4_kernel (4-wave, two workgroups per CU) against the 8-wave mgemm_kernel: GEMM tests with every epilogue
# kind on mg4, then tools/bench_gemm.py with MIA_MG4 unset-equivalent ("") and "all", interleaved.
OUT=gpurun_out/${TAG:-mg4}; mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  MIA_MG4=all timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ast.py -m gpu -x -q \
      --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
SHAPES=${SHAPES:-"fc1.fwd fc2.dgrad proj.fwd fc2.fwd qkv.fwd fc1.dgrad qkv.dgrad proj.dgrad"}
for i in 1 2; do
  for v in "" all; do
    echo "== MIA_MG4='$v' $i" >> $OUT/ab.log
    MIA_MG4=$v REPS=10 timeout -k 10 200 python -u tools/bench_gemm.py $SHAPES >> $OUT/ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu $OUT/ab.log
