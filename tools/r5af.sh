set -o pipefail
mkdir -p gpurun_out/r5ag
timeout -k 10 200 python -u tools/bench_pool.py > gpurun_out/r5ag/r2.log 2>&1 &&
for v in r1 f1 f2; do MIAUDIO_LIB=$PWD/tools/probe/libpool_$v.so timeout -k 10 200 python -u tools/bench_pool.py > gpurun_out/r5ag/$v.log 2>&1 || exit 1; done
