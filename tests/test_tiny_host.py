"""Host layout of the packed degree <= 2 tail (tiny.py) that the fused
launch's tiny-row kernels read (include/kgx.h, kgx_spmm_gemm_ex2): built from
a synthetic degree-descending schedule on the CPU and unpacked again."""

from types import SimpleNamespace

import numpy as np
import torch

from keras_geometric_amd import tiny


def _schedule(n_rows=9000, seed=0, weighted=True):
    """A degree-descending item list {row, begin, end, -1} over a CSR whose
    tail has degree-2, degree-1 and degree-0 rows (plus a few long rows)."""
    rng = np.random.default_rng(seed)
    deg = np.concatenate([np.full(40, 9), np.full(3000, 2), np.full(5000, 1), np.full(n_rows - 8040, 0)])
    rows = rng.permutation(n_rows)
    rowptr = np.zeros(n_rows + 1, np.int64)  # CSR offsets in row-id order
    deg_by_row = np.zeros(n_rows, np.int64)
    deg_by_row[rows] = deg
    rowptr[1:] = np.cumsum(deg_by_row)
    items = np.stack([rows, rowptr[rows], rowptr[rows] + deg, np.full(n_rows, -1)], 1)
    col = rng.integers(0, n_rows, rowptr[-1])
    g = SimpleNamespace(items=torch.from_numpy(items).to(torch.int32), n_items=n_rows, n_long=40,
                        col=torch.from_numpy(col).to(torch.int32),
                        w=torch.from_numpy(rng.standard_normal(rowptr[-1]).astype(np.float32)) if weighted else None)
    return g, items, col


def test_tiny_pack_layout_roundtrip():
    g, items, col = _schedule()
    pack, tw, start, n2 = tiny.tiny_pack(g)
    assert pack is not None and start == 40 and n2 == 3000
    n = g.n_items - start
    assert pack.numel() == tiny.pack_numel(n, n2) and tuple(tw.shape) == (n, 2)
    rec, w = tiny.records(pack, tw, n, n2)
    t = items[start:]
    d = t[:, 2] - t[:, 1]
    np.testing.assert_array_equal(rec[:, 0].numpy(), t[:, 0])
    np.testing.assert_array_equal(rec[:, 1].numpy(), d)
    has = d > 0
    np.testing.assert_array_equal(rec[has, 2].numpy(), col[t[has, 1]])
    two = d == 2
    np.testing.assert_array_equal(rec[two, 3].numpy(), col[t[two, 1] + 1])
    one = d == 1
    np.testing.assert_array_equal(rec[one, 3].numpy(), rec[one, 2].numpy())  # col1 = col0 below degree 2
    ww = g.w.numpy()
    np.testing.assert_array_equal(w[has, 0].numpy(), ww[t[has, 1]])
    np.testing.assert_array_equal(w[two, 1].numpy(), ww[t[two, 1] + 1])
    assert (w[~has].numpy() == 0).all() and (w[one, 1].numpy() == 0).all()
    # every source index the kernels gather is a valid row
    assert int(rec[:, 2].min()) >= 0 and int(rec[:, 3].min()) >= 0


def test_tiny_pack_unweighted_and_unsorted():
    g, items, _ = _schedule(weighted=False, seed=1)
    pack, tw, start, n2 = tiny.tiny_pack(g)
    assert tw is None and n2 == 3000
    # a tail not in degree-descending order: every record takes the two-edge kernel
    g2, items2, _ = _schedule(seed=2)
    perm = np.concatenate([np.arange(40), 40 + np.random.default_rng(3).permutation(len(items2) - 40)])
    g2.items = g2.items[perm]
    pack2, tw2, start2, n2b = tiny.tiny_pack(g2)
    n = g2.n_items - start2
    assert n2b == n
    rec, _ = tiny.records(pack2, tw2, n, n2b)
    t = items2[perm][start2:]
    np.testing.assert_array_equal(rec[:, 1].numpy(), t[:, 2] - t[:, 1])
