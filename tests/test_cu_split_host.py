"""Host logic of the CU-split launches (ops._fused_cu_split / ops._f256_cu_split,
ops._split_allowed) and the ABI flag (KGX_FUSED_CU_SPLIT in include/kgx.h, the
Python constant).  No GPU: which launches ask for the split, and the overrides."""

import re
from pathlib import Path

import pytest

from keras_geometric_amd import _native as nat
from keras_geometric_amd import ops

ROOT = Path(__file__).resolve().parents[1]


def test_flag_matches_header():
    text = (ROOT / "include" / "kgx.h").read_text()
    m = re.search(r"KGX_FUSED_CU_SPLIT\s*=\s*(\d+)", text)
    assert m and int(m.group(1)) == nat.FUSED_CU_SPLIT == 16


@pytest.mark.parametrize("env", [None, "0", "8"])
def test_fused_rule_and_overrides(monkeypatch, env):
    if env is None:
        monkeypatch.delenv("KGX_FUSED_CU_SPLIT", raising=False)
    else:
        monkeypatch.setenv("KGX_FUSED_CU_SPLIT", env)
    ns = ops._fused_cu_split(110_000_000, 8_600_000)      # the north star's schedule
    small = ops._fused_cu_split(11_000_000, 860_000)      # C2
    if env is None:
        assert ns and not small
    elif env == "0":
        assert not ns and not small
    else:
        assert ns and small  # forced
    assert not ops._fused_cu_split(110_000_000, 0)  # nothing to put on the tail CUs


@pytest.mark.parametrize("env", [None, "0", "8"])
def test_f256_model_and_overrides(monkeypatch, env):
    if env is None:
        monkeypatch.delenv("KGX_F256_CU_SPLIT", raising=False)
    else:
        monkeypatch.setenv("KGX_F256_CU_SPLIT", env)
    c4 = ops._f256_cu_split(100_000_000, 7_460_000)       # C4: the tail is a quarter of the time
    tail_heavy = ops._f256_cu_split(100_000_000, 20_000_000)
    tiny = ops._f256_cu_split(1_000_000, 70_000)
    if env is None:
        assert c4 and not tail_heavy and not tiny
    elif env == "0":
        assert not (c4 or tail_heavy or tiny)
    else:
        assert c4 and tail_heavy and tiny


def test_split_off_while_sharing(monkeypatch):
    monkeypatch.delenv("KGX_CU_SPLIT_SHARED", raising=False)
    assert ops._split_allowed()
    with ops.sharing_gpu():
        assert not ops._split_allowed()
        monkeypatch.setenv("KGX_CU_SPLIT_SHARED", "1")
        assert ops._split_allowed()
    assert ops._split_allowed()


def test_split_off_in_the_backward_pass(monkeypatch):
    """The training backward's transposed pass runs one-stream (ops._unsplit), unless
    KGX_BWD_CU_SPLIT=1; the flag is restored on exit, nested or not."""
    monkeypatch.delenv("KGX_CU_SPLIT_SHARED", raising=False)
    monkeypatch.delenv("KGX_BWD_CU_SPLIT", raising=False)
    assert ops._split_allowed()
    with ops._unsplit():
        assert not ops._split_allowed()
        with ops._unsplit():
            assert not ops._split_allowed()
        assert not ops._split_allowed()
    assert ops._split_allowed()
    monkeypatch.setenv("KGX_BWD_CU_SPLIT", "1")
    with ops._unsplit():
        assert ops._split_allowed()


def test_sharing_flag_is_per_thread():
    """Threaded ranks (one process) enter and leave their passes' sharing_gpu
    contexts in any interleaving: the flag is per host thread, so no thread's
    exit leaves another's (or the next caller's) launches flagged."""
    import threading

    a_in, b_in, a_out = threading.Event(), threading.Event(), threading.Event()
    seen = {}

    def rank_a():
        with ops.sharing_gpu():
            a_in.set()
            b_in.wait(5)
            seen["a_inside"] = ops._share_gpu()
        a_out.set()
        seen["a_after"] = ops._share_gpu()

    def rank_b():
        a_in.wait(5)
        with ops.sharing_gpu():
            b_in.set()
            a_out.wait(5)  # A leaves while B is still inside
            seen["b_inside"] = ops._share_gpu()
        seen["b_after"] = ops._share_gpu()

    ts = [threading.Thread(target=rank_a), threading.Thread(target=rank_b)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert seen == {"a_inside": True, "a_after": False, "b_inside": True, "b_after": False}
    assert not ops._share_gpu()


@pytest.mark.parametrize("cus,xccs,arch,ok", [
    (256, 8, b"gfx950:sramecc+:xnack-", True),  # MI355X, SPX: the validated layout
    (256, 8, b"gfx950", True),
    (32, 1, b"gfx950:sramecc+:xnack-", False),  # CPX partition: one XCD per device
    (128, 4, b"gfx950", False),  # DPX
    (240, 8, b"gfx950", False),  # a harvested part
    (304, 8, b"gfx942:sramecc+:xnack-", False),  # MI300X
    (256, 8, b"gfx942", False),
    (256, 8, None, False),
])
def test_cu_split_layout_decision(cus, xccs, arch, ok):
    """The library's fallback decision (kgx_cu_split_layout_ok, kgx_internal.h
    cu_split_layout_ok): split only on the layout it was validated on."""
    assert nat.lib().kgx_cu_split_layout_ok(cus, xccs, arch) == int(ok)


@pytest.mark.parametrize("val,per32", [("8", 8), (" 16 ", 16), ("0", 0), ("32", 0), ("40", 0), ("-3", 0),
                                       ("abc", 0), ("", 0)])
def test_override_parsed_like_the_library(monkeypatch, val, per32):
    """KGX_FUSED_CU_SPLIT / KGX_F256_CU_SPLIT: the Python rule asks for (and counts)
    a split only for values the library runs split (1..31)."""
    monkeypatch.setenv("KGX_FUSED_CU_SPLIT", val)
    monkeypatch.setenv("KGX_F256_CU_SPLIT", val)
    assert ops._per32_override("KGX_FUSED_CU_SPLIT") == per32
    assert ops._fused_cu_split(110_000_000, 8_600_000) == (per32 > 0)
    assert ops._f256_cu_split(100_000_000, 7_460_000) == (per32 > 0)


def test_split_off_on_unvalidated_device(monkeypatch):
    import torch

    monkeypatch.delenv("KGX_CU_SPLIT_SHARED", raising=False)
    monkeypatch.setattr(ops, "_DEVICE_SPLIT_OK", {0: False, 1: True})
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    assert not ops._split_allowed(torch.device("cuda", 0))
    assert not ops._split_allowed(torch.device("cuda", 1))  # not the current device: the library runs it unsplit
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 1)
    assert ops._split_allowed(torch.device("cuda", 1))
