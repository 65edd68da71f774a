"""Summarise rocprofv3 PMC passes into the per-launch HBM traffic bench.py reports.

  python tools/pmc_summary.py FETCH_CSV WRITE_CSV OUT_JSON [--config ns]

FETCH_CSV / WRITE_CSV are rocprofv3 `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
counter_collection.csv files of the same bench.py command.  Per kernel the
median over dispatches is taken (the first launches include graph-build
effects).  Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM /
rocprofv3): both counters are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of 16-B-per-lane reads (TCC_EA0_RDREQ x 64 B for 128-B requests), so it
is doubled -- verified for this kernel family's row-gather pattern by the
calibration in tools/exp_agg.py `calib`.
WRITE_SIZE is exact for 16-B-per-lane stores.

Every kernel entry carries a hash of ITS sources: the .hip file that defines
it plus the csrc/ headers that file includes (kernel_source_hash); bench.py attaches
the traffic only when the hash of each kernel it reports matches the sources
it runs, so a stale profile is never reported against a changed kernel, and an
edit to an unrelated kernel's file does not invalidate it.
"""

from __future__ import annotations

import csv
import hashlib
import json
import re
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "keras-geometric_amd" / "csrc"




def source_hash() -> str:
    """Hash of every kernel source (kept for the profile's header; per-kernel
    validity uses kernel_source_hash)."""
    h = hashlib.sha256()
    for p in sorted(CSRC.glob("*")):
        if p.suffix in (".hip", ".cpp", ".h"):
            h.update(p.name.encode())
            h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _closure(path: Path, seen: set) -> None:
    """path and the kernel-side headers it includes (csrc/), transitively.  The
    public ABI header include/kgx.h is left out: its declarations and comments
    change with the boundary, not with the kernels' code."""
    if path in seen or not path.exists():
        return
    seen.add(path)
    for inc in re.findall(r'#include\s+"([^"]+)"', path.read_text()):
        if (CSRC / inc).exists():
            _closure(CSRC / inc, seen)


def kernel_file(kernel: str) -> Path | None:
    """The .hip file whose __global__ function is named `kernel` (a short name)."""
    pat = re.compile(r"__global__[^;{]*?\b" + re.escape(kernel) + r"\s*\(", re.S)
    for p in sorted(CSRC.glob("*.hip")):
        if pat.search(p.read_text()):
            return p
    return None


def kernel_source_hash(kernel: str) -> str | None:
    """Hash of the source file defining `kernel` and the headers it includes."""
    f = kernel_file(kernel)
    if f is None:
        return None
    files: set = set()
    _closure(f, files)
    h = hashlib.sha256()
    for p in sorted(files, key=lambda q: q.name):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def per_kernel(path: str, counter: str) -> dict[str, float]:
    vals: dict[str, list[float]] = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def short(name: str) -> str:
    base = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return base.split("::")[-1].split("<")[0]


def main() -> None:
    fetch_csv, write_csv, out = sys.argv[1:4]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "ns"
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        fk, wk = fetch.get(name), write.get(name)
        t = (2 * fk * 1024 if fk is not None else 0) + (wk * 1024 if wk is not None else 0)
        k = kernels.get(short(name))
        if k is not None:  # several instantiations launched per step (e.g. the tiny kernel's two parts): summed
            k["kernel"] += " + " + name
            k["traffic_bytes_per_launch"] += t
            continue
        kernels[short(name)] = {
            "kernel": name,
            "source_hash": kernel_source_hash(short(name)),
            "fetch_size_kib_median": fk,
            "write_size_kib_median": wk,
            "traffic_bytes_per_launch": t,
        }
    json.dump({"config": config, "source_hash": source_hash(), "correction": "FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024",
               "kernels": kernels}, open(out, "w"), indent=1)
    print(json.dumps({k: v["traffic_bytes_per_launch"] / 1e9 for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
