#!/bin/bash
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ast.py tests/test_gpu_fullsize.py -k "attention or attn" > gpurun_out/attn_rev_tests.log 2>&1 || { tail -40 gpurun_out/attn_rev_tests.log; exit 1; }
tail -2 gpurun_out/attn_rev_tests.log
bash tools/attn_ab.sh ${1:-attnhead} > /dev/null
grep -v amdgpu gpurun_out/attnab/ab.log | grep -E "==|round"
