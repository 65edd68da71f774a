"""HBM traffic of one TRAINING step from rocprofv3 PMC passes (the training
step launches the same kernel names for the forward and the transposed dx pass,
so per-kernel medians, tools/pmc_summary.py, would mix the two).

  python tools/pmc_step.py FETCH_CSV WRITE_CSV OUT_JSON --per-step N --steps S

Takes the last S x N dispatches of each pass (the timed steps of a
`bench.py --train --steps S` run profiled with a kernel-include regex that keeps
exactly N launches per step), sums FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024
(the corrections tools/pmc_summary.py documents) and divides by S.  Every kernel
seen carries its source hash (pmc_summary.kernel_source_hash) so bench.py
attaches the number only to the sources it was measured from."""

import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import pmc_summary as ps  # noqa: E402


def dispatches(path: str, counter: str) -> list[tuple[int, str, float]]:
    out: dict[int, list] = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            if d not in out:
                out[d] = [r["Kernel_Name"], 0.0]
            out[d][1] += float(r["Counter_Value"])  # summed over the counter's instances
    return [(d, v[0], v[1]) for d, v in sorted(out.items())]


def main() -> None:
    fetch_csv, write_csv, out = sys.argv[1:4]
    n = int(sys.argv[sys.argv.index("--per-step") + 1])
    steps = int(sys.argv[sys.argv.index("--steps") + 1])
    fe = dispatches(fetch_csv, "FETCH_SIZE")[-n * steps:]
    wr = dispatches(write_csv, "WRITE_SIZE")[-n * steps:]
    names_f = [ps.short(k) for _, k, _ in fe]
    names_w = [ps.short(k) for _, k, _ in wr]
    if names_f != names_w or len(fe) != n * steps or names_f[:n] * steps != names_f:
        raise SystemExit(f"the two passes' last {n * steps} dispatches do not repeat one step of {n}: {names_f[:n]}")
    traffic = (sum(2 * v * 1024 for _, _, v in fe) + sum(v * 1024 for _, _, v in wr)) / steps
    kernels = {k: ps.kernel_source_hash(k) for k in sorted(set(names_f))}
    json.dump({"step_kernels": names_f[:n], "kernels": {k: {"source_hash": h} for k, h in kernels.items()},
               "steps": steps, "traffic_bytes_per_step": traffic,
               "correction": "FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024"}, open(out, "w"), indent=1)
    print(json.dumps({"traffic_GB_per_step": traffic / 1e9, "step_kernels": names_f[:n]}))


if __name__ == "__main__":
    main()
