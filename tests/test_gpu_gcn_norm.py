"""GCN normalisation bit-exact to the reference's arithmetic.

utils/main.py:20-33: degrees = segment_sum(ones, target); dinv =
power(add(degrees, 1e-12), -0.5); dinv[isinf] = 0; norm_e = dinv[dst] *
dinv[src].  On the Keras-torch backend `power` is torch.pow(Tensor, 0-dim
Tensor), i.e. ATen's vectorised powf (not correctly rounded for some degrees).
kgx takes dinv from a table of exactly those values (graph.gcn_dinv_table,
kgx_csr_build2), so dinv and every edge norm must equal the oracle's bit for
bit.

One caveat is the reference's own: ATen's vector loop hands the last few
elements of each thread's chunk of the degree vector to libm's scalar powf,
so which nodes get the scalar value depends on the thread count of the
machine running it.  The bitwise comparison therefore evaluates the oracle
expression with every element on the vector path (one thread, length padded
to a whole vector), and the default multi-threaded oracle is compared with
the rest held to <= 1 ulp at <= 64 nodes per thread.
"""

import numpy as np
import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd import graph as G
from keras_geometric_amd import synthetic
from oracle import keras_torch as K
from oracle import reference as R

pytestmark = [pytest.mark.gpu]


@pytest.fixture(autouse=True)
def _release():
    yield
    G.clear_cache()
    torch.cuda.empty_cache()


def _oracle_dinv_vector_path(degrees: torch.Tensor) -> torch.Tensor:
    """utils/main.py:24-27 on the oracle's ops, every element on ATen's vector path."""
    n = degrees.numel()
    pad = (-n) % 64
    d = torch.cat([degrees, torch.ones(pad, dtype=degrees.dtype)])
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        out = []
        for i in range(0, d.numel(), 16384):  # below ATen's grain size: one chunk, no scalar leftovers
            out.append(K.power(K.add(d[i:i + 16384], 1e-12), -0.5))
        dinv = torch.cat(out)[:n]
    finally:
        torch.set_num_threads(threads)
    return K.where(K.isinf(dinv), torch.zeros_like(dinv), dinv)


def _ulp_diff(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return (a.view(torch.int32).long() - b.view(torch.int32).long()).abs()


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_c2_gcn_norm_bit_exact(dev):
    n, e = 1_000_000, 10_000_000
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    ei_l = R.add_self_loops(ei.cpu(), n)
    ones = torch.ones(ei_l.shape[1], dtype=torch.float32)
    degrees = K.segment_sum(ones, ei_l[1], n)  # utils/main.py:23-24
    assert torch.equal(degrees, g.deg.cpu().float())
    dinv_v = _oracle_dinv_vector_path(degrees)
    assert torch.equal(g.dinv.cpu(), dinv_v)
    # norm in CSR order == the oracle's per-input-edge norm taken at each slot's input edge id
    src, dst = ei_l[0], ei_l[1]
    norm_v = K.multiply(K.take(dinv_v, dst, axis=0), K.take(dinv_v, src, axis=0))
    assert torch.equal(g.w.cpu(), norm_v[g.eid.cpu().long()])
    # the reference exactly as it runs here (multi-threaded): equal but for the scalar leftovers
    norm_ref = R.compute_gcn_normalization(ei_l, n)
    diff = _ulp_diff(g.w.cpu(), norm_ref[g.eid.cpu().long()])
    dinv_ref = K.power(K.add(degrees, 1e-12), -0.5)
    dd = _ulp_diff(g.dinv.cpu(), dinv_ref)
    assert int(dd.max()) <= 1 and int((dd > 0).sum()) <= 64 * torch.get_num_threads(), int((dd > 0).sum())
    bad_nodes = torch.nonzero(dd > 0).flatten()
    touched = torch.isin(dst[g.eid.cpu().long()], bad_nodes) | torch.isin(src[g.eid.cpu().long()], bad_nodes)
    assert int(diff[~touched].max()) == 0 and int(diff.max()) <= 2


def test_rmat_small_norm_equals_golden(golden, dev):
    """The committed fixture's norm (tests/golden/make_golden.py: the oracle's
    compute_gcn_normalization over 2048 nodes, one chunk of whole vectors)."""
    gz = golden("rmat_small")
    ei = torch.from_numpy(gz["edge_index"]).to(dev).int()
    n = int(gz["x"].shape[0])
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    assert torch.equal(g.w.cpu(), torch.from_numpy(gz["gcn_norm_loops"])[g.eid.cpu().long()])


def test_dinv_table_grows(dev):
    """A degree past the cached table: kgx_csr_build2 reports the miss and the
    build redoes dinv / w from a longer table (graph.build_csr)."""
    G._DINV_TABLES.clear()
    n, hub = 6000, 5000  # one row of degree 5001 (with its loop) > the initial 4096 entries
    src = torch.arange(hub, dtype=torch.int32)
    dst = torch.zeros(hub, dtype=torch.int32)
    ei = torch.stack([src, dst]).to(dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    assert G._DINV_TABLES[str(dev)].numel() >= hub + 2
    ei_l = R.add_self_loops(ei.cpu().long(), n)
    degrees = K.segment_sum(torch.ones(ei_l.shape[1]), ei_l[1], n)
    dinv_v = _oracle_dinv_vector_path(degrees)
    assert torch.equal(g.dinv.cpu(), dinv_v)
    norm_v = K.multiply(K.take(dinv_v, ei_l[1], axis=0), K.take(dinv_v, ei_l[0], axis=0))
    assert torch.equal(g.w.cpu(), norm_v[g.eid.cpu().long()])


def _integer_inputs(n, f_in, f_out, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randint(-4, 5, (n, f_in), generator=gen).float()
    W = torch.randint(-3, 4, (f_in, f_out), generator=gen).float()
    b = torch.randint(-2, 3, (f_out,), generator=gen).float() / 4
    return x, W, b


@pytest.mark.parametrize("self_loops", [True, False])
@pytest.mark.parametrize("fixture", ["toy_gcn", "rmat_small", "cora_like"])
def test_gcn_exact_layer_bit_identical(fixture, self_loops, golden, dev):
    """GCNConv end to end in EXACT mode == the oracle's gcn_conv.py:275-364, bit for
    bit.  Integer-valued x and W make x_j W exact in fp32 whatever the GEMM's
    summation order (the reference's per-edge CPU matmul vs kgx's node-level
    MFMA product), so every remaining operation -- degree, dinv, norm, the
    message's * norm, the edge-ordered segment sum, + bias -- is compared."""
    gz = golden(fixture)
    ei = torch.from_numpy(gz["edge_index"]).long()
    n = int((gz["x"] if "x" in gz else gz["x_packed"]).shape[0])
    x, W, b = _integer_inputs(n, 16, 8, 7)
    layer = kgx.GCNConv(8, add_self_loops=self_loops, exact=True)
    with torch.no_grad():
        layer([x.to(dev), ei.to(dev)])
        layer.set_weights([W.numpy(), b.numpy()])
        y = layer([x.to(dev), ei.to(dev)]).cpu()
    ref = R.gcn_forward(x, ei, W, b, add_self_loops_=self_loops)
    assert torch.equal(y, ref), float((y - ref).abs().max())
