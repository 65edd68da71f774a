# Round 6: CU census per split size (why splits other than 8 / 16 of every 32 ran slowly).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6census2
mkdir -p $O
timeout -k 10 300 python -u tools/exp_cu_census.py > $O/census.jsonl 2> $O/err.log || exit $?
