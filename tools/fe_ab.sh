set -e
mkdir -p gpurun_out/feab

LOGMEL_LIBS=tools/probe/libmia_logmel_old.so BATCH=256 timeout -k 10 120 python -u tools/bench_logmel.py > gpurun_out/feab/logmel.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_logmel.py tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py > gpurun_out/feab/tests.log 2>&1
