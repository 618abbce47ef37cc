set -o pipefail
mkdir -p gpurun_out/r5aw
timeout -k 10 400 python -u tools/bench_gemm.py fc1.fwd:gelu_save_d fc1.fwd:gelu_save_d+mxq fc1.fwd@mx:gelu_save_d fc1.fwd@mx:gelu_save_d+mxq fc1.fwd@mx:plain fc1.fwd:plain fc2.dgrad:dmul fc2.dgrad@mx:dmul fc2.dgrad@mx:dmul+mxq fc2.dgrad@mx:plain fc2.fwd fc2.fwd@mx qkv.fwd qkv.fwd@mx fc1.dgrad fc1.dgrad@mx > gpurun_out/r5aw/gemm.log 2>&1
