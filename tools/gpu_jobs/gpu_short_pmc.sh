# SQ PMC passes (one rocprofv3 run per pass) on the fused GCN short-row kernel (tools/exp_short.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/spmc
PASS_A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
PASS_B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES"
PASS_C="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVES"
i=0
for P in "$PASS_A" "$PASS_B" "$PASS_C"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d gpurun_out/spmc/p$i -o run \
    --kernel-include-regex "spmm_gemm_(short_)?kernel" -- python3 tools/exp_short.py > gpurun_out/spmc/p$i.log 2>&1 || echo "pass $i failed rc=$?"
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/spmc/p*/run_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = "short" if "short" in r["Kernel_Name"] else "long"
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f, k, {c: round(sum(v) / max(1, len(set(v)) and len(v)), 1) for c, v in d.items()})
PY
