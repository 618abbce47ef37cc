#!/bin/bash
# dense GEMM K-loop without the vmcnt(0) stall (asm transposed reads, LDS scratch in the staging array):
# GEMM/optim/e2e parity, then both bench legs
OUT=gpurun_out/r2w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_optim.py tests/test_gpu_e2e_bf16.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 900 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2w/bench.json'))
print(d['value'], d['ms_per_step']); print({k:v['ms'] for k,v in d['kernels'].items()})
a=d['ast']; print(a['value'], a['ms_per_step']); print({k:(v['ms'], round(v['tflops'])) for k,v in a['kernels'].items()})
PY
