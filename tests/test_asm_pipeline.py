"""Wait-counter and LDS hand-off hazards, checked on the compiled gfx950 ISA (CPU).

Several kernels keep memory operations in flight on purpose: spmm_hub_kernel
and dense_kernel issue their loads as inline asm with counted `s_waitcnt
vmcnt(N)` (hipcc cannot see those registers are still being written, so a
copy or reuse it places while a load is in flight reads or corrupts data),
and the tiny-row / 256-wide fused kernels hand tiles between waves through
LDS with `lds_barrier()` (an lgkmcnt-only wait: gathers stay in flight across
the barrier).  tools/isa_hazard_check.py models the vmcnt / lgkmcnt queues of
one wave over each kernel's control-flow graph (branch conditions from scalar
flags, loops to a fixed point) and reports any read or overwrite of a
register a pending load will still write, and any LDS op in flight at an
s_barrier.

This compiles the kernel sources for gfx950 to assembly and requires:
  * no register hazard in any checked instantiation;
  * no LDS op in flight at a barrier, except in spmm_hub_kernel, whose
    consumers leave their ring reads in flight across a barrier (the producers
    overwrite that ring slot two barriers later, spmm.hip hub_barrier_reader)
    and whose claim of the next item is read after the next hub_barrier.
It found two real hazards in dense_kernel's producer epilogue (DESIGN.md §4,
"ISA hazard check"), since fixed.
"""

import contextlib
import io
import multiprocessing
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "keras-geometric_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
sys.path.insert(0, str(ROOT / "tools"))

import isa_hazard_check as H  # noqa: E402

# (source, extra flags, kernel-name patterns checked; [] = every kernel in the file)
SOURCES = {
    "spmm": ("spmm.hip", ["-std=c++17"], ["spmm_hub_kernel", "spmm_kernel", "spmm_short_kernel"]),
    # every instantiation of the fused 128-wide kernels: sum, mean, max, min, weighted
    # or not, one or two tables, narrow or not; short and tiny tails, fix-ups
    "spmm_gemm": ("spmm_gemm.hip", ["-std=c++17"], ["ILi0E", "ILi1E", "ILi2E", "ILi3E"]),
    "spmm_gemm256": ("spmm_gemm256.hip", ["-std=c++17"], []),
    "dense": ("dense.hip", ["-std=c++20", "-fno-slp-vectorize"], ["dense_kernel"]),
}
BARRIER_HANDOFF_OK = ("spmm_hub_kernel",)
# held to the exec-masked row-load rule too (tools/isa_hazard_check.py): every
# gather and descriptor load of the 128-wide fused kernels is issued with full exec
EXEC_RULE = ("spmm_gemm_kernel", "spmm_gemm_short_kernel", "spmm_gemm_tiny_kernel")


def _check(job):
    name, body = job
    sys.path.insert(0, str(ROOT / "tools"))
    import isa_hazard_check as HC

    with contextlib.redirect_stdout(io.StringIO()):
        return name, HC.check_kernel(body, name, 0, exec_rule=any(p in name for p in EXEC_RULE))


def _compile(tmp: Path, key: str) -> str:
    src, flags, _ = SOURCES[key]
    out = tmp / f"{key}.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-ffp-contract=off", *flags, f"-I{ROOT / 'include'}",
                    f"-I{CSRC}", "-x", "hip", "--cuda-device-only", "-S", str(CSRC / src), "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


@pytest.mark.timeout(900)
@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_kernels_have_no_inflight_hazards(tmp_path):
    with ThreadPoolExecutor(len(SOURCES)) as ex:
        asm = dict(zip(SOURCES, ex.map(lambda k: _compile(tmp_path, k), SOURCES)))
    jobs = [(name, body) for key, text in asm.items() for name, body in H.kernels(text, SOURCES[key][2])
            if "rocprim" not in name]
    ctx = multiprocessing.get_context("spawn")  # never fork a process that may hold torch threads
    with ctx.Pool(min(8, os.cpu_count() or 1)) as pool:
        results = pool.map(_check, jobs, chunksize=1)
    checked, bad = len(jobs), []
    for name, found in results:
        for (line, why), ins in found:
            if "at s_barrier" in why and any(p in name for p in BARRIER_HANDOFF_OK):
                continue
            bad.append(f"{name}: line {line}: {why}: {ins}")
    assert checked >= 200, checked  # every family present
    assert sum(any(p in name for p in EXEC_RULE) for name, _ in jobs) >= 90
    assert not bad, "\n".join(bad[:20])


def test_checker_flags_planted_hazards():
    """The model itself: a weakened vmcnt wait, a dropped lgkmcnt before a
    barrier, and a register reused under a pending load are all reported."""
    base = [
        "k:",
        "global_load_dwordx4 v[0:3], v[10:11], off",
        "global_load_dwordx4 v[4:7], v[10:11], off offset:16",
        "s_waitcnt vmcnt(1)",
        "v_add_f32_e32 v8, v0, v1",  # v[0:3] landed (one newer op may still fly)
        "ds_write_b32 v9, v8",
        "s_waitcnt lgkmcnt(0)",
        "s_barrier",
        "s_waitcnt vmcnt(0)",
        "v_add_f32_e32 v8, v4, v5",
        "s_endpgm",
    ]

    def hazards(lines):
        with contextlib.redirect_stdout(io.StringIO()):
            return [why for (_, why), _ in H.check_kernel(lines, "t", 0)]

    assert hazards(base) == []
    weak = list(base)
    weak[3] = "s_waitcnt vmcnt(2)"
    assert any("read of a register" in w for w in hazards(weak))
    nolgkm = [l for l in base if "lgkmcnt" not in l]
    assert any("LDS write in flight at s_barrier" in w for w in hazards(nolgkm))
    reuse = list(base)
    reuse.insert(4, "v_mov_b32_e32 v5, 0")  # v5 belongs to the load still in flight
    assert any("write to a register a pending load" in w for w in hazards(reuse))
    # a branch that skips the newer load: the wait no longer covers the older one
    branchy = ["k:", "global_load_dword v0, v[10:11], off", "s_cbranch_scc1 .LBB0_1",
               "global_load_dword v1, v[10:11], off", ".LBB0_1:", "s_waitcnt vmcnt(1)",
               "v_mov_b32_e32 v2, v0", "s_endpgm"]
    assert any("read of a register" in w for w in hazards(branchy))


def test_exec_rule_flags_masked_prefetch():
    """The exec-masked row-load rule: a 16-byte gather issued inside an
    s_and_saveexec region and folded after the region's join (the round-4
    fused prefetch, `if (u < pn) vload(pv[u])`) is reported; the same gather
    issued after the join (full exec, the zero-row form) is not; a gather
    consumed inside its region, or joined only out of an inner loop, is not."""
    masked = [
        "k:",
        "s_and_saveexec_b64 s[0:1], vcc",
        "s_cbranch_execz .LBB0_1",
        "global_load_dwordx4 v[4:7], v[10:11], off",
        ".LBB0_1:",
        "s_or_b64 exec, exec, s[0:1]",
        "s_waitcnt vmcnt(0)",
        "v_mul_f32_e32 v8, v4, v9",
        "s_endpgm",
    ]

    def hazards(lines):
        with contextlib.redirect_stdout(io.StringIO()):
            return [why for (_, why), _ in H.check_kernel(lines, "t", 0, exec_rule=True)]

    assert any("exec-masked" in w for w in hazards(masked))
    # off by default (the hand-pipelined kernels are checked for wait counts only)
    with contextlib.redirect_stdout(io.StringIO()):
        assert H.check_kernel(masked, "t", 0) == []
    full = ["k:", "s_and_saveexec_b64 s[0:1], vcc", "s_cbranch_execz .LBB0_1", "v_mov_b32_e32 v10, v12",
            ".LBB0_1:", "s_or_b64 exec, exec, s[0:1]", "global_load_dwordx4 v[4:7], v[10:11], off",
            "s_waitcnt vmcnt(0)", "v_mul_f32_e32 v8, v4, v9", "s_endpgm"]
    assert hazards(full) == []
    inside = masked[:4] + ["s_waitcnt vmcnt(0)", "v_mul_f32_e32 v8, v4, v9"] + masked[4:6] + ["s_endpgm"]
    assert hazards(inside) == []
    # a divergent loop inside the region: its exit join does not leave the load's region
    loop = ["k:", "s_and_saveexec_b64 s[0:1], vcc", "global_load_dwordx4 v[4:7], v[10:11], off",
            "s_mov_b64 s[2:3], 0", ".LBB0_2:", "s_or_b64 s[2:3], vcc, s[2:3]", "s_andn2_b64 exec, exec, s[2:3]",
            "s_cbranch_execnz .LBB0_2", "s_or_b64 exec, exec, s[2:3]", "s_waitcnt vmcnt(0)",
            "v_mul_f32_e32 v8, v4, v9", "s_or_b64 exec, exec, s[0:1]", "s_endpgm"]
    assert hazards(loop) == []
