# SQ PMC passes on the NS aggregation kernels (spmm_kernel and the fused spmm_gemm_kernel; tools/exp_agg.py both)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/npmc
PASS_A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PASS_B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES"
PASS_C="TCC_HIT TCC_MISS TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ"
i=0
for P in "$PASS_A" "$PASS_B" "$PASS_C"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d gpurun_out/npmc/p$i -o run \
    --kernel-include-regex 'spmm' -- python3 tools/exp_agg.py both > gpurun_out/npmc/p$i.log 2>&1 || exit $?
done
