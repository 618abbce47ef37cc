#!/bin/bash
# coalesced two-pass column sums behind the LN backward and the dGELU pass: AST tests, gemm colsum
# tests, the bf16 end-to-end steps, then the AST bench leg
OUT=gpurun_out/r2s9; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_ast.py tests/test_gpu_e2e_bf16.py tests/test_gpu_gemm.py -x -q -k "not conv and not fe_ and not rowconv and not rowwgrad and not tap and not wgrad8 and not trunk" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --model ast --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2s9/bench.json'))
d=d.get('ast', d)
print(d['value'], d['ms_per_step']); print({k:v['ms'] for k,v in d['kernels'].items()})
PY
