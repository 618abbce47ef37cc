set -o pipefail
mkdir -p gpurun_out/r5bm
timeout -k 10 600 python -u -m pytest tests/test_gpu_norm.py -k "pool_raw_stats or raw_winners" -x -v --timeout 300 --timeout-method thread > gpurun_out/r5bm/tests.log 2>&1 &&
MIA_POOL_RAW_THREAD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_norm.py -k "pool_raw_stats" -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bm/tests_old.log 2>&1 ;
timeout -k 10 900 python -u -m pytest tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py tests/test_gpu_train_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bm/tests2.log 2>&1 &&
for r in 1 2; do
  MIA_POOL_RAW_THREAD=1 timeout -k 10 300 python -u bench.py --model envnet --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5bm/old$r.json 2>/dev/null &&
  timeout -k 10 300 python -u bench.py --model envnet --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5bm/new$r.json 2>/dev/null || exit 1
done
