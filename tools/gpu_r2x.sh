#!/bin/bash
# re-entry check of HEAD on a fresh box: whole GPU suite, smoke, default bench line (both legs)
OUT=gpurun_out/r2x; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/r2x/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['frontend_path']['frac']); print({k:v['ms'] for k,v in d['kernels'].items()})
a=d['ast']; print(a['value'], a['ms_per_step']); print({k:(v['ms'], round(v['tflops'])) for k,v in a['kernels'].items()})
PY
