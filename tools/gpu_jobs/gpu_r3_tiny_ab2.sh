# round 3: degree-1 tiny kernel, committed form (ab_head/, a `git archive HEAD` copy built in place) against the
# working tree: NS bench under rocprofv3 kernel stats, interleaved twice
set -o pipefail
mkdir -p gpurun_out/r3ab2
export TMPDIR=/tmp
ROOTD=$PWD
for r in 1 2; do
  for t in head new; do
    d=$ROOTD; [ $t = head ] && d=$ROOTD/ab_head
    (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTD/gpurun_out/r3ab2/${t}_$r -o run \
      -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $ROOTD/gpurun_out/r3ab2/${t}_$r.json 2> $ROOTD/gpurun_out/r3ab2/${t}_$r.err) || exit $?
    f=$(find gpurun_out/r3ab2/${t}_$r -name '*kernel_stats.csv' | head -n 1)
    echo "== $t round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3ab2/${t}_$r.json)"
    grep -E 'spmm_gemm' "$f" | awk -F'","' '{print $1}' | cut -c1-10 > /dev/null
    python3 - "$f" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if 'spmm_gemm' in row['Name']:
        print(f"  {row['Name'][30:95]:65s} calls {row['Calls']:>4} avg {float(row['AverageNs'])/1e6:.3f} ms")
PY
  done
done
