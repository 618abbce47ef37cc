#!/bin/bash
# Round-4 GPU pass (through gpurun from the repo root): new tests first, then the whole -m gpu suite,
# smoke and the default bench line.  Each GPU step has its own limit; the chain stops at a failure
# that is not a plain test failure (a timeout / abort / fault ends the call).
OUT=gpurun_out/r4
mkdir -p $OUT
# heartbeat: long oracle runs at the benched sizes print nothing for minutes (each step still has its
# own timeout); the file under gpurun_out/ shows the harness the call is alive
( while sleep 45; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
export MIOPEN_FIND_MODE=FAST  # the oracle's torch convs on the GPU: no exhaustive solver search
STAGES=${STAGES:-"new tests smoke bench"}
NEW=${NEW:-"tests/test_gpu_deferred_wgrad.py tests/test_gpu_ast.py::test_attn_saved_q_equals_plain tests/test_gpu_gemm.py::test_mgemm_ragged_n_not_multiple_of_8 tests/test_gpu_train_script.py::test_train_script_config5_ast_fp8_urbansound8k tests/test_gpu_fullsize.py"}
for s in $STAGES; do
  case $s in
    new)
      timeout -k 10 900 python -u -m pytest $NEW -m gpu -v -s --timeout 400 --timeout-method thread > $OUT/new_tests.log 2>&1
      rc=$? ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1
      rc=$? ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$? ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
      rc=$? ;;
    *)
      echo "unknown stage $s"; exit 2 ;;
  esac
  echo "stage $s rc=$rc"
  # 1 = some tests failed (keep going); anything else non-zero (timeout 124/137, abort 134, segv 139) stops
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
