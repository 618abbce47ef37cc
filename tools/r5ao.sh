set -o pipefail
mkdir -p gpurun_out/r5ao
CONV8_LIBS=tools/probe/libconv8_ref.so timeout -k 10 300 python -u tools/bench_conv8.py > gpurun_out/r5ao/bench.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_envnet.py -x -q --timeout 120 --timeout-method thread -k "conv8 or trunk" > gpurun_out/r5ao/tests.log 2>&1
