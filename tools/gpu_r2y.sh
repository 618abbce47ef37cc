#!/bin/bash
# AST backward with the bias gradients folded (LN backward column sums, attention dK/dV/dQ column
# sums): AST parity tests, bf16 e2e step, AST bench leg
OUT=gpurun_out/r2y; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ast.py tests/test_gpu_e2e_bf16.py tests/test_gpu_gemm.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --model ast --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2y/bench.json'))
a=d.get('ast', d); print(a['value'], a['ms_per_step']); print({k:(v['ms'], round(v['tflops'])) for k,v in a['kernels'].items()})
PY
