set -o pipefail
mkdir -p gpurun_out/r5av
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8_ast.py tests/test_gpu_ast.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5av/tests.log 2>&1 &&
for v in fc2,fc1,proj fc2,fc1,proj,qkv; do
  MIA_MX_DGRAD=$v timeout -k 10 400 python -u bench.py --model ast-fp8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5av/b_$v.json 2> gpurun_out/r5av/b_$v.err || exit 1
done
timeout -k 10 400 python -u bench.py --model ast --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5av/b_bf16.json 2> gpurun_out/r5av/b_bf16.err
