#!/bin/bash
# log-mel balanced mel projection: parity tests + AST bench leg; then the hipBLASLt BGRADB probe
OUT=gpurun_out/r2t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_logmel.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --model ast --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2t/bench.json')); a=d.get('ast',d)
print(a['value'], a['ms_per_step'], a['kernels']['logmel.fwd'])
PY

