"""The hub kernel's inline-asm load pipeline, checked on the compiled ISA (CPU).

spmm_hub_kernel (EXACT rows of degree >= 2048) issues its gathers as inline
asm with counted vmcnt waits, so hipcc cannot see that those registers are
still being written; a register copy or reuse the allocator places while a
load is in flight would read or corrupt data (a debug variant that broke the
invariant faulted on the GPU with a memory-aperture violation).  This
compiles csrc/spmm.hip for gfx950 to assembly and runs
tools/asm_vmcnt_check.py over every instantiation of the kernel.
"""

import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "keras-geometric_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_hub_kernel_has_no_inflight_register_hazards(tmp_path):
    asm = tmp_path / "spmm.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    f"-I{ROOT / 'include'}", f"-I{CSRC}", "-x", "hip", "--cuda-device-only", "-S",
                    str(CSRC / "spmm.hip"), "-o", str(asm)], check=True, capture_output=True)
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "asm_vmcnt_check.py"), str(asm), "spmm_hub_kernel"],
                       capture_output=True, text=True)
    assert r.stdout.count("hazards 0") == 32, r.stdout[-3000:]
    assert r.returncode == 0, r.stdout[-3000:]
