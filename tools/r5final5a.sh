set -o pipefail
mkdir -p gpurun_out/r5final5
( while sleep 45; do date +%T >> gpurun_out/r5final5/hb_tests.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5final5/gpu_tests.log 2>&1 &&
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final5/smoke.log 2>&1
