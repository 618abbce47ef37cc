set -o pipefail
mkdir -p gpurun_out/r5bf
timeout -k 10 600 python -u -m pytest tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py tests/test_gpu_train_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "not ast" > gpurun_out/r5bf/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model envnet --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5bf/bench.json 2> gpurun_out/r5bf/bench.err
