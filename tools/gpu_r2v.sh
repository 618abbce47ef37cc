#!/bin/bash
# FC wgrad sum-of-squares epilogue + clip/Adam pre-partials: parity tests, EnvNet e2e, EnvNet bench
OUT=gpurun_out/r2v; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_optim.py tests/test_gpu_e2e_bf16.py tests/test_gpu_envnet.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --model envnet --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2v/bench.json'))
print(d['value'], d['ms_per_step'], d['frontend_path']); print({k:v['ms'] for k,v in d['kernels'].items()})
PY
