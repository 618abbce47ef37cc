set -o pipefail
mkdir -p gpurun_out/r5an
LOGMEL_LIBS=tools/probe/libmia_lmold.so,tools/probe/libmia_lmt3.so,tools/probe/libmia_lmfullns.so,tools/probe/libmia_lmnone.so,tools/probe/libmia_lmnonens.so,tools/probe/libmia_lmnonenl.so,tools/probe/libmia_lmnonenlns.so timeout -k 10 300 python -u tools/bench_logmel.py > gpurun_out/r5an/bench.log 2>&1
