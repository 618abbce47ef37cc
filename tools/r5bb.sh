set -o pipefail
mkdir -p gpurun_out/r5bb
timeout -k 10 300 python -u tools/bench_gemm.py fc2.dgrad:dmul fc2.dgrad:dmul_nocs fc2.dgrad:dmul fc2.dgrad:dmul_nocs fc2.dgrad:plain > gpurun_out/r5bb/g.log 2>&1
