#!/bin/bash
OUT=gpurun_out/r2f; mkdir -p $OUT
timeout -k 10 120 python -u tools/diag_logmel_zero.py > $OUT/diag.log 2>&1; rc=$?; cat $OUT/diag.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_ast.py tests/test_gpu_logmel.py tests/test_gpu_e2e_bf16.py -s > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|\[ast\]" $OUT/tests.log | tail -12
[ $rc -gt 1 ] && exit $rc
BATCH=256 timeout -k 10 300 python -u tools/bench_attn.py > $OUT/attn.log 2>&1 || exit $?
cat $OUT/attn.log
BATCH=64 bash tools/attn_pmc.sh r2f/attn || exit $?
timeout -k 10 300 python -u bench.py --model ast --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_ast.json 2> $OUT/bench_ast.err; rc=$?
echo "bench rc=$rc"; python -c "
import json; d=json.load(open('$OUT/bench_ast.json')); print(d['value'], d['ms_per_step']); print({k:(round(v['ms'],3), round(v['tflops'],1)) for k,v in d['kernels'].items()})"
exit $rc
