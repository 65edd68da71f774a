#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over `exp_agg.py both`
# (NS unfused spmm + fused GCN kernel).  Usage: bash tools/gpu_jobs/gpu_pmc.sh
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run \
    --kernel-include-regex "spmm" -- python3 tools/exp_agg.py both > gpurun_out/pmc/g$i.log 2>&1 || exit $?
done
