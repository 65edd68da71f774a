# Round 5: NS fused op with the tiny-row launches forked beside the main and
# short-row kernels (KGX_FUSED_FORK=1) against the sequential order, interleaved
# bench lines (same box), then the round-5 profiles (profiles/r05/command_pmc.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
for i in 1 2 3; do
  for f in 0 1 2; do
    KGX_FUSED_FORK=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
      > gpurun_out/r5b/ns_fork$f.$i.json 2> gpurun_out/r5b/ns_fork$f.$i.err || exit $?
  done
done
python - <<'PY'
import json, glob
for f in (0, 1, 2):
    ms = [json.loads(open(p).read().strip().splitlines()[-1])["ms_per_step"] for p in sorted(glob.glob(f"gpurun_out/r5b/ns_fork{f}.*.json"))]
    print("KGX_FUSED_FORK", f, "ms", ms)
PY
