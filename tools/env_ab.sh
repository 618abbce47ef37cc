#!/bin/bash
# EnvNet probe A/B (temporary): tests on each probe, then the step with per-kernel probes
OUT=gpurun_out/envab; mkdir -p $OUT
for v in "$@"; do
  MIAUDIO_LIB=$(realpath tools/probe/libmia_$v.so) timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_envnet.py tests/test_gpu_deferred_wgrad.py tests/test_gpu_norm.py > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $OUT/tests_$v.log)"
done
rm -rf gpurun_out/abm
bash tools/ab_multi.sh "--model envnet --steps 30 --warmup 5 --no-cpu-baseline --probe ${PROBES:-t0a.wgrad,fc1.fwd,fc1.dgrad,fc2.fwd}" base "$@"
