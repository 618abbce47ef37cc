#!/bin/bash
# clip + Adam with the tensors ordered largest first: optimizer tests, EnvNet e2e step, EnvNet bench
OUT=gpurun_out/r2s10; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_envnet.py tests/test_gpu_e2e_bf16.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --model envnet --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2s10/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac']); print({k:v['ms'] for k,v in d['kernels'].items()})
PY
