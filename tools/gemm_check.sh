mkdir -p gpurun_out/gemm
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -q -x -k "dense" --timeout 120 --timeout-method thread > gpurun_out/gemm/t.log 2>&1
MIA_DGEMM256=0 timeout -k 10 120 python -u tools/bench_gemm.py > gpurun_out/gemm/old.log 2>&1
MIA_DGEMM256=1 timeout -k 10 120 python -u tools/bench_gemm.py > gpurun_out/gemm/new.log 2>&1
echo done
