set -o pipefail
mkdir -p gpurun_out/r5bh
timeout -k 10 600 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_mx.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bh/tests.log 2>&1 &&
LN_LIBS=tools/probe/libnorm_ref.so timeout -k 10 300 python -u tools/bench_ln.py > gpurun_out/r5bh/ln.log 2>&1
