# Round 3: SQ counters of the fused-256 kernels (tiny tail and main) on the C4 graph.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/f256pmc
PASS_A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
PASS_B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE"
i=0
for P in "$PASS_A" "$PASS_B"; do
  i=$((i+1))
  KGX_EXP_UNFUSED=0 timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d gpurun_out/f256pmc/p$i -o run \
    --kernel-include-regex 'gemm256' -- python3 tools/exp_f256.py > gpurun_out/f256pmc/p$i.log 2>&1 || exit $?
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/f256pmc/p*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = ('tiny' if 'tiny' in r['Kernel_Name'] else 'fixup' if 'fixup' in r['Kernel_Name'] else 'main')
        acc[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
    for (k, c), v in sorted(acc.items()):
        v.sort()
        print(k, c, v[len(v) // 2])
PY
