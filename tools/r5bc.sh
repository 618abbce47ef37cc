set -o pipefail
mkdir -p gpurun_out/r5bd
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_gemm.py fc1.fwd:gelu_save_d+mxq fc1.fwd@mx:gelu_save_d+mxq fc2.dgrad@mx:dmul+mxq > gpurun_out/r5bd/dpp$r.log 2>&1 &&
MIAUDIO_LIB=$PWD/tools/probe/libmia_mxshfl.so timeout -k 10 300 python -u tools/bench_gemm.py fc1.fwd:gelu_save_d+mxq fc1.fwd@mx:gelu_save_d+mxq fc2.dgrad@mx:dmul+mxq > gpurun_out/r5bd/shfl$r.log 2>&1 || exit 1
done
