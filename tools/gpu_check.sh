#!/bin/bash
# One GPU-box pass (run through gpurun from the repo root):
#   gpu parity tests -> smoke -> EnvNet bench (with cpu_baseline) -> AST bench
# Each GPU step has its own time limit; the chain stops at the first failure.
set -e
OUT=gpurun_out/check
mkdir -p $OUT
STAGES=${STAGES:-"tests smoke envnet ast"}
for s in $STAGES; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
          > $OUT/gpu_tests.log 2>&1 ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    envnet)
      timeout -k 10 300 python -u bench.py > $OUT/bench_envnet.log 2>&1 ;;
    ast)
      timeout -k 10 300 python -u bench.py --model ast --no-cpu-baseline > $OUT/bench_ast.log 2>&1 ;;
  esac
  echo "stage $s ok"
done
