# Single-hub-row scaling: kernel time vs degree, source range and width.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hubscan
i=0
for cfg in "1 138539" "1 69270" "1 138539 1000" "1 138539 1000000 64" "1 138539 1000000 256" "4 138539"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hubscan/c$i -o run -- python3 tools/exp_hub_synth.py $cfg > gpurun_out/hubscan/c$i.json 2>&1 || exit 1
  python3 - "$i" "$cfg" <<'PY'
import csv, sys
i, cfg = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(f"gpurun_out/hubscan/c{i}/run_kernel_stats.csv")))
print(cfg, [(r["Name"].split("namespace)::")[-1][:18], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows if "spmm" in r["Name"]], flush=True)
PY
done
