set -o pipefail
mkdir -p gpurun_out/r5ah
timeout -k 10 400 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py tests/test_gpu_train_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ah/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model envnet --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5ah/bench.log 2>&1
