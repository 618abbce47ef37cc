set -o pipefail
mkdir -p gpurun_out/r5bk
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py tests/test_gpu_train_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "not ast" > gpurun_out/r5bk/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model envnet --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5bk/new$r.json 2>/dev/null &&
  MIA_W2_DROPCOPY=1 timeout -k 10 300 python -u bench.py --model envnet --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5bk/old$r.json 2>/dev/null || exit 1
done
