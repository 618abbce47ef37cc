set -o pipefail
mkdir -p gpurun_out/r5az
REPS=30 timeout -k 10 300 python -u tools/bench_gemm.py qkv.fwd fc1.fwd:gelu_save_d > gpurun_out/r5az/g0.log 2>&1 &&
GAP_MB=512 REPS=30 timeout -k 10 300 python -u tools/bench_gemm.py qkv.fwd fc1.fwd:gelu_save_d > gpurun_out/r5az/g512.log 2>&1 &&
GAP_MB=2048 REPS=30 timeout -k 10 300 python -u tools/bench_gemm.py qkv.fwd fc1.fwd:gelu_save_d > gpurun_out/r5az/g2048.log 2>&1
