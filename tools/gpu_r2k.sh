#!/bin/bash
# hipBLASLt plain-GEMM path: GEMM tests, per-shape tile vs library timing, AST bench
OUT=gpurun_out/r2k; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" $OUT/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
TOKENS=421120 timeout -k 10 300 python -u tools/bench_gemm.py > $OUT/gemm.log 2>&1 || { tail $OUT/gemm.log; exit 1; }
cat $OUT/gemm.log
timeout -k 10 400 python -u bench.py --model ast --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_ast.json 2> $OUT/bench_ast.err; rc=$?
echo "bench rc=$rc"; python -c "
import json; d=json.load(open('$OUT/bench_ast.json')); a=d.get('ast', d); print(a['value'], a['ms_per_step']); print({k:(round(v['ms'],3), round(v.get('tflops',0),1)) for k,v in a['kernels'].items()})"
exit $rc
