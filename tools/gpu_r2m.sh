#!/bin/bash
OUT=gpurun_out/r2m; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_ast.py tests/test_gpu_e2e_bf16.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" $OUT/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
bash tools/trace_only.sh r2m_ast "--model ast --steps 3 --warmup 2 --no-cpu-baseline" || exit $?
python tools/trace_by_kernel.py gpurun_out/prof_r2m_ast/trace/run_kernel_trace.csv adam_kernel 16
grep -o '"value": [0-9.]*' gpurun_out/prof_r2m_ast/bench_trace.log | head -2
