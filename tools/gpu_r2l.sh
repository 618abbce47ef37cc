#!/bin/bash
# AST kernel trace (hipBLASLt path)
bash tools/trace_only.sh r2l_ast "--model ast --steps 3 --warmup 2 --no-cpu-baseline" || exit $?
python tools/trace_by_kernel.py gpurun_out/prof_r2l_ast/trace/run_kernel_trace.csv adam_kernel 45
