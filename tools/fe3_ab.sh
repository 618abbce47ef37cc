#!/bin/bash
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_norm.py tests/test_gpu_envnet.py > gpurun_out/fe3_tests.log 2>&1 || { tail -30 gpurun_out/fe3_tests.log; exit 1; }
tail -2 gpurun_out/fe3_tests.log
bash tools/ab_multi.sh "--model envnet --steps 20 --warmup 5 --no-cpu-baseline" base fehead
