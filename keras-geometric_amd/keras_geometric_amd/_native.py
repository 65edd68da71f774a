"""ctypes binding of libkgx.so (the C-ABI declared in include/kgx.h).

The library is the product path: there is no CPU or pure-PyTorch fallback.
If it is missing, or a kernel is asked to run on a CPU tensor, the call fails
loudly.  torch is imported first so that the HIP runtime torch ships is the one
libkgx binds to (both use the soname libamdhip64.so.7), which makes torch's
device pointers and streams valid inside the library.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_PKG_ROOT = Path(__file__).resolve().parent.parent  # keras-geometric_amd/
LIB_PATH = Path(os.environ.get("KGX_LIB", _PKG_ROOT / "lib" / "libkgx.so"))

KGX_OK, KGX_ERR_ARG, KGX_ERR_HIP, KGX_ERR_INDEX, KGX_ERR_UNSUPPORTED = range(5)
SUM, MEAN, MAX, MIN, STD = range(5)
EPI_NONE, EPI_BIAS, EPI_GIN, EPI_RAW, EPI_ACCUM = range(5)
FUSED_PRE_GIN, FUSED_ACCUMULATE, FUSED_SHARE_GPU, FUSED_RELU, FUSED_CU_SPLIT = 1, 2, 4, 8, 16
CSR_SELF_LOOPS, CSR_SEGMENT_ONLY, CSR_GCN_NORM = 1, 2, 4
DENSE_RELU, DENSE_ACCUMULATE = 1, 2
DENSE_MAX_K, DENSE_MAX_N = 256, 256

REDUCE_IDS = {"sum": SUM, "mean": MEAN, "max": MAX, "min": MIN, "std": STD}

_i32p = ctypes.c_void_p
_f32p = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int

# name -> argtypes (every entry point returns int unless listed in _RESTYPES)
_SIGNATURES = {
    "kgx_version": [],
    "kgx_last_error": [],
    "kgx_csr_workspace_bytes": [_i64, _i64, _int, ctypes.POINTER(ctypes.c_size_t)],
    "kgx_csr_build": [
        _i32p, _i32p, _i64, _i64, _i64, _int,
        _i32p, _i32p, _i32p, _i32p, _f32p, _f32p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
    ],
    "kgx_csr_build2": [
        _i32p, _i32p, _i64, _i64, _i64, _int,
        _i32p, _i32p, _i32p, _i32p, _f32p, _f32p, _f32p, _i64,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
    ],
    "kgx_gcn_dinv": [_i32p, _i64, _f32p, ctypes.c_void_p],
    "kgx_cu_split_layout_ok": [_int, _int, ctypes.c_char_p],
    "kgx_schedule_suffixes": [_i32p, _i64, _int, _int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                              ctypes.c_void_p],
    "kgx_tiny_pack": [_i32p, _i64, _i64, _i32p, _f32p, _i64, _i32p, _f32p, ctypes.c_void_p,
                      ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p],
    "kgx_gemm_tn_workspace_bytes": [_i64, _i64, _i64, ctypes.POINTER(ctypes.c_size_t)],
    "kgx_gemm_tn": [_i64, _f32p, _i64, _i64, _f32p, _i64, _i64, _f32p, _i64, _f32p, ctypes.c_void_p,
                    ctypes.c_size_t, ctypes.c_void_p],
    "kgx_cu_split_supported": [_int],
    "kgx_cu_split_census": [_int, _i64, _i32p, _i32p, ctypes.POINTER(ctypes.c_int), ctypes.c_void_p],
    "kgx_gcn_dinv_table": [_i32p, _i64, _f32p, _i64, _f32p, ctypes.c_void_p],
    "kgx_gcn_edge_norm": [_i32p, _i32p, _i64, _f32p, _f32p, _f32p, ctypes.c_void_p],
    "kgx_schedule_workspace_bytes": [_i64, ctypes.POINTER(ctypes.c_size_t)],
    "kgx_schedule_build": [
        _i32p, _i64, ctypes.c_int32, _i32p, _i32p, _i64, _i32p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
    ],
    "kgx_spmm": [
        _int, _int, _i32p, _i32p, _i64, _i32p, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _i64, _f32p, _i64,
        _f32p, _f32p, _i64, ctypes.c_float, _i32p, ctypes.c_float, ctypes.c_uint64, _f32p, ctypes.c_void_p,
    ],
    "kgx_spmm_ex": [
        _int, _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _i64, _f32p, _i64,
        _f32p, _f32p, _i64, ctypes.c_float, _i32p, ctypes.c_float, ctypes.c_uint64, _f32p, ctypes.c_void_p,
    ],
    "kgx_spmm_ex2": [
        _int, _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _f32p, _i64, _i64, _f32p, _i64,
        _f32p, _f32p, _i64, ctypes.c_float, _i32p, ctypes.c_float, ctypes.c_uint64, _f32p, _i32p, ctypes.c_void_p,
    ],
    "kgx_dropout_mask": [ctypes.c_uint64, ctypes.c_float, _i32p, _i64, _i64, _f32p, ctypes.c_void_p],
    "kgx_spmm_gemm": [
        _int, _i32p, _i32p, _i64, _i32p, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_spmm_gemm_ex": [
        _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_spmm_gemm_ex2": [
        _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i64, _i32p, _f32p, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_spmm_gemm_f256": [
        _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i64, _i32p, _f32p, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_spmm_gemm_f256_ex": [
        _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i64, _i32p, _f32p, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_spmm_gemm_ex3": [
        _int, _i32p, _i32p, _i64, _i32p, _i64, _i64, _i64, _i32p, _f32p, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_spmm_max_backward": [
        _int, _int, _i32p, _i64, _i32p, _f32p, _i64, _i64, _f32p, _i64, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_gatv2_backward": [
        _i32p, _i32p, _i64, _i32p, _i64, _i32p, _i64, _i32p, _f32p, _f32p, _i64, _f32p, _int, _int,
        ctypes.c_float, _f32p, _i64, _f32p, _f32p, _f32p, _i64,
        _i32p, _i32p, _i64, _i32p, _i64, _i32p, _i64, _i32p, _i32p,
        _f32p, _f32p, _i64, _f32p, _f32p, _f32p, _f32p, _i32p, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p,
    ],
    "kgx_gatv2": [
        _i32p, _i32p, _i64, _i32p, _i64, _i32p, _i64,
        _i32p, _f32p, _f32p, _i64, _f32p, _int, _int, ctypes.c_float,
        _f32p, _i64, _f32p, _f32p, _f32p, _i32p, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p,
    ],
    "kgx_dense": [
        _i64, _f32p, _i64, _i64, _f32p, _f32p, _i64, _i64, _f32p, _i64, _f32p, _int, _f32p, _i64, ctypes.c_void_p,
    ],
    "kgx_gather_rows": [_f32p, _i64, _i32p, _i64, _i64, _f32p, _i64, ctypes.c_void_p],
    "kgx_scatter_f32": [_f32p, _i32p, _i64, _f32p, ctypes.c_void_p],
    "kgx_rmat_edges": [
        ctypes.c_uint64, _int, _i64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
        _i64, _i64, _i32p, _i32p, ctypes.c_void_p,
    ],
    "kgx_select_workspace_bytes": [_i64, ctypes.POINTER(ctypes.c_size_t)],
    "kgx_select_dst_range": [
        _i32p, _i32p, _i64, _i64, _i64, _i32p, _i32p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
    ],
}
_RESTYPES = {"kgx_last_error": ctypes.c_char_p}

_lib: ctypes.CDLL | None = None


def lib() -> ctypes.CDLL:
    """Load libkgx.so once; raise if it has not been built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"kgx native library not found at {LIB_PATH}. Build it with "
                "`make -C keras-geometric_amd/csrc` (or __graft_entry__.build())."
            )
        handle = ctypes.CDLL(str(LIB_PATH))
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = handle
    return _lib


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)


def check(rc: int, what: str) -> None:
    if rc == KGX_OK:
        return
    msg = lib().kgx_last_error().decode(errors="replace")
    if rc == KGX_ERR_INDEX:
        raise IndexError(msg)
    if rc in (KGX_ERR_ARG, KGX_ERR_UNSUPPORTED):
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def require_device(*tensors: torch.Tensor | None) -> torch.device:
    """All kernel operands must live on one ROCm device; no host fallback."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "kgx kernels run on MI355X (ROCm) only: got a tensor on "
                f"{t.device}. Move inputs to a cuda device; there is no CPU path."
            )
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"kgx: tensors on different devices ({dev} vs {t.device})")
    if dev is None:
        raise RuntimeError("kgx: no device tensor given")
    return dev


def ptr(t: torch.Tensor | None) -> ctypes.c_void_p | None:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
