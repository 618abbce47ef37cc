# PMC passes over tools/bench_fe.py (run through gpurun from the repo root)
set -e
ROOT=$(pwd)
mkdir -p $ROOT/gpurun_out/fepmc
timeout -k 10 120 python -u tools/bench_fe.py > $ROOT/gpurun_out/fepmc/bench.log 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VALU --kernel-trace --kernel-include-regex feconv --output-format csv -d $ROOT/gpurun_out/fepmc/a -o run -- python3 $ROOT/tools/bench_fe.py > $ROOT/gpurun_out/fepmc/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS --kernel-trace --kernel-include-regex feconv --output-format csv -d $ROOT/gpurun_out/fepmc/b -o run -- python3 $ROOT/tools/bench_fe.py > $ROOT/gpurun_out/fepmc/b.log 2>&1
echo done
