# Round 5: C4 tail (spmm_gemm256_tiny2_kernel) cost decomposition, timing-only
# builds: gathers replaced by cache hits (KGX_T2_NOGATHER), no MFMA phase
# (KGX_T2_NOMFMA), both; interleaved with the shipped build (tools/exp_f256.py
# -> gpurun_out/t2d/ab.log); then two SQ counter passes over the shipped C4
# kernels (-> gpurun_out/t2d/sq{1,2}).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t2d
mkdir -p $O
: > $O/ab.log
for round in 0 1; do
  for lib in main t2nog t2nom t2nogm; do
    if [ $lib = main ]; then L=keras-geometric_amd/lib/libkgx.so; else L=keras-geometric_amd/lib/variants/libkgx_$lib.so; fi
    KGX_EXP_UNFUSED=0 KGX_LIB=$L timeout -k 10 240 python tools/exp_f256.py >> $O/ab.log 2> $O/$lib.err || exit $?
  done
done
PASS_A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
PASS_B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD"
i=0
for P in "$PASS_A" "$PASS_B"; do
  i=$((i+1))
  KGX_EXP_UNFUSED=0 timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/sq$i -o run \
    --kernel-include-regex 'gemm256' -- python3 tools/exp_f256.py > $O/sq$i.log 2>&1 || exit $?
done
