mkdir -p gpurun_out/gemm
export TMPDIR=/tmp
cd /tmp
for v in 0 1; do
MIA_DGEMM256=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS --kernel-trace --kernel-include-regex dgemm --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gemm/pmc$v -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_gemm.py > $GRAFT_REPO_ROOT/gpurun_out/gemm/pmc$v.log 2>&1
done
echo done
