#!/bin/bash
set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_e2e_bf16.py -k "gelu or ast" > gpurun_out/dgelu_tests.log 2>&1 || { tail -30 gpurun_out/dgelu_tests.log; exit 1; }
tail -2 gpurun_out/dgelu_tests.log
SHAPES="fc2.dgrad" bash tools/gemm_ab.sh mghead
