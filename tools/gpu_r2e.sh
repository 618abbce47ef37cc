#!/bin/bash
# one gpurun call: log-mel diagnosis, GPU tests (no -x), attention SQ counters, AST bench
OUT=gpurun_out/r2e; mkdir -p $OUT
timeout -k 10 120 python -u tools/diag_logmel_zero.py > $OUT/diag.log 2>&1; rc=$?; cat $OUT/diag.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_e2e_bf16.py tests/test_gpu_train_script.py tests/test_gpu_logmel.py -s > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -gt 1 ] && exit $rc
BATCH=64 bash tools/attn_pmc.sh r2e/attn || exit $?
timeout -k 10 300 python -u bench.py --model ast --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_ast.json 2> $OUT/bench_ast.err; rc=$?
echo "bench rc=$rc"; head -c 1500 $OUT/bench_ast.json
exit $rc
