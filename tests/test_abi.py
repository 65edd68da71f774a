"""The C-ABI library loads and exports every entry point include/kgx.h declares (CPU)."""

import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "kgx.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(kgx_\w+)\s*\(", text, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from keras_geometric_amd import _native

    return _native.lib()


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "kgx_spmm" in syms and "kgx_csr_build" in syms and "kgx_gatv2" in syms
    assert len(syms) >= 13


def test_every_declared_symbol_is_exported(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"libkgx.so lacks {missing}"


def test_binding_covers_header(lib):
    from keras_geometric_amd import _native

    assert set(declared_symbols()) <= set(_native.exported_symbols())


def test_version_and_error_channel(lib):
    assert lib.kgx_version() == 1
    rc = lib.kgx_spmm(99, 0, None, None, 1, None, 0, None, 0, None, None, None, 1, 1, None, 1, None, None, 0,
                      1.0, None, 0.0, 0, None, None)
    assert rc == 1  # KGX_ERR_ARG, no device touched
    assert b"unknown reduce" in lib.kgx_last_error()


def test_argument_validation_without_device(lib):
    from keras_geometric_amd import _native as nat

    # split_len not a power of two
    assert lib.kgx_schedule_build(ctypes.c_void_p(16), 4, 3, None, None, 0, None, None, 0, None, None) == 1
    assert b"power of two" in lib.kgx_last_error()
    # self loops need a square graph
    rc = lib.kgx_csr_build(None, None, 0, 3, 4, nat.CSR_SELF_LOOPS, None, None, None, None, None, None, None, 0,
                           None, None)
    assert rc == 1
    # unsupported GAT shape (too many lanes per row) is reported, not launched
    rc = lib.kgx_gatv2(ctypes.c_void_p(16), ctypes.c_void_p(16), 1, None, 0, None, 0, ctypes.c_void_p(16),
                       ctypes.c_void_p(16), ctypes.c_void_p(16), 64 * 33, ctypes.c_void_p(16), 64, 33, 0.2,
                       ctypes.c_void_p(16), 64 * 33, None, None, None, None, 0.0, 0, None)
    assert rc == 4
    # message dropout only for sums, p in [0, 1)
    rc = lib.kgx_spmm(2, 0, ctypes.c_void_p(16), ctypes.c_void_p(16), 1, None, 0, None, 0, ctypes.c_void_p(16), None,
                      ctypes.c_void_p(16), 4, 4, ctypes.c_void_p(16), 4, None, None, 0, 1.0, ctypes.c_void_p(16), 0.5,
                      1, None, None)
    assert rc == 1 and b"dropout" in lib.kgx_last_error()
    # backward of max/min only; fused accumulate flag validation
    assert lib.kgx_spmm_max_backward(0, 0, None, 0, None, None, 0, 0, None, 0, None, 0, None) == 1
    # rmat argument checks
    assert lib.kgx_rmat_edges(0, 4, 100, 1, 1, 1, 0, 10, None, None, None) == 1


def test_library_refuses_cpu_tensors():
    import torch

    from keras_geometric_amd import _native as nat

    with pytest.raises(RuntimeError, match="no CPU path"):
        nat.require_device(torch.zeros(3))
