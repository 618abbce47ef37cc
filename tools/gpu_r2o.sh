#!/bin/bash
OUT=gpurun_out/r2o; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm.py -k "bgrad or plain" tests/test_gpu_ast.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" $OUT/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
bash tools/trace_only.sh r2o_ast "--model ast --steps 3 --warmup 2 --no-cpu-baseline" || exit $?
python tools/trace_by_kernel.py gpurun_out/prof_r2o_ast/trace/run_kernel_trace.csv adam_kernel 16
grep -o '"value": [0-9.]*' gpurun_out/prof_r2o_ast/bench_trace.log | head -2
