#!/bin/bash
# pooled-backward raw-winner gather: parity tests, then an EnvNet kernel trace
OUT=gpurun_out/r2j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_norm.py tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
bash tools/trace_only.sh r2j_envnet "--model envnet --steps 5 --warmup 2 --no-cpu-baseline" || exit $?
python tools/trace_by_kernel.py gpurun_out/prof_r2j_envnet/trace/run_kernel_trace.csv adam_kernel 40 pool_bwd_sparse
tail -2 gpurun_out/prof_r2j_envnet/bench_trace.log
