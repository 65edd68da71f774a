# Round 6: kgx_gemm_tn LDS form counters (SQ wait / issue / MFMA busy / LDS, clock).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6tnpmc
mkdir -p $O
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --output-format csv -d $O/p1 -o tn -- python -u $GRAFT_REPO_ROOT/tools/exp_gemm_tn.py --reps 3 > $O/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES \
  --output-format csv -d $O/p2 -o tn -- python -u $GRAFT_REPO_ROOT/tools/exp_gemm_tn.py --reps 3 > $O/p2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o tn -- python -u $GRAFT_REPO_ROOT/tools/exp_gemm_tn.py --reps 3 > $O/p3.log 2>&1 || exit $?
