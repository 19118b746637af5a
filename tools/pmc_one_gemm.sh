export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
for v in ${VARIANTS:-7 12}; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc1/v$v -o run -- python3 tools/gemm_bench.py one 2304 512 2048 0 1 0 $v > gpurun_out/pmc1/v$v.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM --kernel-trace --output-format csv -d gpurun_out/pmc1/w$v -o run -- python3 tools/gemm_bench.py one 2304 512 2048 0 1 0 $v > gpurun_out/pmc1/w$v.log 2>&1 || exit 1
done
echo ok
