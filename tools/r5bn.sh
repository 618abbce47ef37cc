set -o pipefail
mkdir -p gpurun_out/r5bn
timeout -k 10 600 python -u -m pytest tests/test_gpu_norm.py -k "conv3_wgrad" -x -v --timeout 300 --timeout-method thread > gpurun_out/r5bn/tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py tests/test_gpu_train_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bn/tests2.log 2>&1 &&
for r in 1 2; do
  MIA_C3_BNSEP=1 timeout -k 10 300 python -u bench.py --model envnet --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5bn/old$r.json 2>/dev/null &&
  timeout -k 10 300 python -u bench.py --model envnet --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5bn/new$r.json 2>/dev/null || exit 1
done
