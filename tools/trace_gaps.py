"""Idle time between kernels in a rocprofv3 --kernel-trace CSV (a measurement helper).

  python tools/trace_gaps.py gpurun_out/r4/c5_trace [--last 20]

Sorts the dispatches by start time and reports, over the last N dispatches of
the run (the timed steps), the busy time (union of kernel intervals), the idle
gaps between them, and the kernels by total time: a layer's wall time minus its
kernels' busy time is what runs on the host or waits between launches.
"""

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(path: str):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=0, help="only the last N dispatches (0: all)")
    ap.add_argument("--match", default="", help="start the window at the first dispatch whose name contains this")
    args = ap.parse_args()
    rows = load(args.path)
    if args.last:
        rows = rows[-args.last:]
    if args.match:
        i = next((k for k, r in enumerate(rows) if args.match in r[2]), 0)
        rows = rows[i:]
    busy, gaps, end = 0, [], None
    per = defaultdict(float)
    for s, e, name in rows:
        per[name.replace("(anonymous namespace)::", "").split("(")[0][-60:]] += (e - s) / 1e6
        if end is None or s >= end:
            if end is not None:
                gaps.append((s - end) / 1e6)
            busy += e - s
            end = e
        elif e > end:
            busy += e - end
            end = e
    span = (rows[-1][1] - rows[0][0]) / 1e6 if rows else 0.0
    print(json.dumps({"dispatches": len(rows), "span_ms": span, "busy_ms": busy / 1e6, "idle_ms": sum(gaps),
                      "largest_gaps_ms": sorted(gaps, reverse=True)[:8],
                      "kernels_ms": dict(sorted(per.items(), key=lambda kv: -kv[1])[:12])}, indent=1))


if __name__ == "__main__":
    main()
