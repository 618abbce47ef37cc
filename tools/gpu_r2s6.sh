#!/bin/bash
# GELU passes with blocks dividing the column groups: epilogue parity tests, then the AST bench leg
OUT=gpurun_out/r2s6; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q -k "plain_gemm or colsum or epilogues" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --model ast --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2s6/bench.json'))
d=d.get('ast', d)
print(d['value'], d['ms_per_step']); print({k:v['ms'] for k,v in d['kernels'].items()})
PY
