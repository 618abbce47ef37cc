set -o pipefail
mkdir -p gpurun_out/r5bi
BATCH=256 ATTN_LIBS=tools/probe/libattn_ref.so timeout -k 10 400 python -u tools/bench_attn.py > gpurun_out/r5bi/attn.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_ast.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "attention or attn" > gpurun_out/r5bi/tests.log 2>&1
