# PMC passes (one rocprofv3 run per pass, kernel-include dense) on the C4 dense shape for the main library and variants.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dpmc
(cd /tmp && timeout -k 10 120 rocprofv3 -L) > gpurun_out/dpmc/counters.txt 2>&1 || echo "counter list failed"
PASS_A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
PASS_B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES"
for v in main "$@"; do
  if [ "$v" = main ]; then lib=keras-geometric_amd/lib/libkgx.so; else lib=keras-geometric_amd/lib/variants/libkgx_$v.so; fi
  i=0
  for P in "$PASS_A" "$PASS_B"; do
    i=$((i+1))
    KGX_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/dpmc/${v}_$i -o run \
      --kernel-include-regex dense -- python3 tools/bench_dense.py --only ${ONLY:-C4} --reps 3 > gpurun_out/dpmc/${v}_$i.log 2>&1 || exit $?
  done
done
