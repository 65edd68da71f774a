"""Training-mode dropout on the propagate path: GCNConv message dropout
(gcn_conv.py:237-242) and GATv2Conv attention dropout (gatv2_conv.py:252-253).

Keras draws its masks from its own RNG, so no mask can match the reference
bit for bit; what is pinned is the arithmetic given a mask.  kgx's mask is a
pure function of (seed, input edge id, column/head) -- kgx_dropout_mask
exposes it -- and the layers' outputs and gradients must equal the oracle's
forward with that same mask applied where the reference applies Dropout."""

import numpy as np
import pytest
import torch

from keras_geometric_amd import ops as kops
from keras_geometric_amd.layers import GATv2Conv, GCNConv
from oracle import keras_torch as K
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for

pytestmark = pytest.mark.gpu
T = torch.from_numpy


def rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else b
    return float((np.abs(a.astype(np.float64) - b) / np.maximum(1.0, np.abs(b))).max())


def test_mask_statistics(dev):
    keys = torch.arange(200_000, dtype=torch.int32, device=dev)
    for p in (0.1, 0.5, 0.9):
        m = kops.dropout_mask(7, p, keys, 16).cpu().numpy()
        vals = np.unique(m)
        keep = np.float32(1.0) / (np.float32(1.0) - np.float32(p))  # 1/(1-p) in fp32, as the kernel
        assert set(vals.tolist()) <= {0.0, float(keep)}
        assert abs((m == 0).mean() - p) < 3e-3
    a = kops.dropout_mask(7, 0.5, keys, 16)
    assert torch.equal(a, kops.dropout_mask(7, 0.5, keys, 16))  # deterministic
    assert not torch.equal(a, kops.dropout_mask(8, 0.5, keys, 16))  # seed matters


def _gcn_oracle(x, ei, W, b, mask):
    """gcn_forward with Dropout(x_j W) = (x_j W) * mask, mask per input edge (self loops last)."""
    n = x.shape[0]
    eil = R.add_self_loops(ei, n)
    w = R.compute_gcn_normalization(eil, n)
    x_j = K.take(x, eil[0], axis=0)
    msg = (torch.matmul(x_j, W) * mask) * torch.unsqueeze(w, 1)
    return K.add(R.aggregate("sum", msg, eil[1], n), b)


@pytest.mark.parametrize("exact", [True, False])
def test_gcn_message_dropout_forward_backward(dev, exact):
    N, Fi, Fo, E, p = 1200, 32, 24, 12000, 0.3
    s, d = rmat_edges(40, scale_for(N), N, 0, E)
    ei = np.stack([s, d]).astype(np.int32)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((N, Fi)).astype(np.float32)
    layer = GCNConv(Fo, dropout_rate=p, exact=exact)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    W = (rng.standard_normal((Fi, Fo)) * 0.2).astype(np.float32)
    b = rng.standard_normal(Fo).astype(np.float32)
    layer.set_weights([W, b])
    torch.manual_seed(123)
    seed = int(torch.randint(0, 2**62, (1,)).item())  # the draw the layer makes
    torch.manual_seed(123)
    y = layer([xd, T(ei).to(dev)], training=True)
    gout = rng.standard_normal((N, Fo)).astype(np.float32)
    y.backward(T(gout).to(dev))
    mask = kops.dropout_mask(seed, p, torch.arange(E + N, dtype=torch.int32, device=dev), Fo).cpu()
    xr, Wr, br = T(x).requires_grad_(True), T(W).requires_grad_(True), T(b).requires_grad_(True)
    yr = _gcn_oracle(xr, T(ei), Wr, br, mask)
    yr.backward(T(gout))
    assert rel(y, yr) <= 1e-5
    assert rel(xd.grad, xr.grad) <= 1e-5
    assert rel(layer.kernel.grad, Wr.grad) <= 1e-5 * np.sqrt(N)
    assert (mask == 0).float().mean().item() == pytest.approx(p, abs=0.02)
    # inference (training=False) ignores the dropout rate
    y0 = layer([xd, T(ei).to(dev)]).detach()
    assert rel(y0, R.gcn_forward(T(x), T(ei), T(W), T(b))) <= 1e-5


def _gat_oracle(x, ei, kernel, att, bias, heads, mask):
    """gatv2_forward with Dropout(alpha) = alpha * mask[edge, head]."""
    n = x.shape[0]
    eil = R.add_self_loops(K.cast(ei, torch.int32), n)
    C = kernel.shape[1] // heads
    e = eil.shape[1]
    h = torch.matmul(x, kernel).reshape(n, heads, C)
    src, dst = eil[0], eil[1]
    h_j, h_i = K.take(h, src, axis=0), K.take(h, dst, axis=0)
    z = K.leaky_relu(K.add(h_i, h_j), 0.2)
    scores = torch.sum(K.multiply(z, att), dim=-1)
    mx = K.segment_max(scores, dst, n)
    ex = torch.exp(scores - K.take(mx, dst, axis=0))
    ssum = K.segment_sum(ex, dst, n)
    alpha = K.divide(ex, K.add(K.take(ssum, dst, axis=0), 1e-10)) * mask
    aggr = K.segment_sum((torch.unsqueeze(alpha, -1) * h_j).reshape(e, heads * C), dst, n)
    return aggr + bias


def test_gat_attention_dropout_forward_backward(dev):
    N, Fi, H, C, E, p = 800, 16, 4, 8, 7000, 0.25
    s, d = rmat_edges(41, scale_for(N), N, 0, E)
    ei = np.stack([s, d]).astype(np.int32)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((N, Fi)).astype(np.float32)
    layer = GATv2Conv(C, heads=H, dropout=p, exact=True)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    with torch.no_grad():
        layer.bias.copy_(T(rng.standard_normal(H * C).astype(np.float32)))
    kern, att, bias = (t.detach().cpu() for t in (layer.linear_transform.kernel, layer.att, layer.bias))
    torch.manual_seed(5)
    seed = int(torch.randint(0, 2**62, (1,)).item())
    torch.manual_seed(5)
    y = layer([xd, T(ei).to(dev)], training=True)
    gout = rng.standard_normal((N, H * C)).astype(np.float32)
    y.backward(T(gout).to(dev))
    mask = kops.dropout_mask(seed, p, torch.arange(E + N, dtype=torch.int32, device=dev), H).cpu()
    xr = T(x).requires_grad_(True)
    kr, ar, br = (t.clone().requires_grad_(True) for t in (kern, att, bias))
    yr = _gat_oracle(xr, T(ei), kr, ar, br, H, mask)
    yr.backward(T(gout))
    assert rel(y, yr) <= 1e-5
    assert rel(xd.grad, xr.grad) <= 1e-5
    assert rel(layer.att.grad, ar.grad) <= 1e-5 * np.sqrt(N)
    assert rel(layer.linear_transform.kernel.grad, kr.grad) <= 1e-5 * np.sqrt(N)


@pytest.mark.parametrize("aggregator", ["mean", "max", "sum", "pooling"])
def test_sage_message_dropout_forward_backward(dev, aggregator):
    """SAGEConv training-mode Dropout(x_j) (sage_conv.py:280-298; for 'pooling'
    before the pool MLP): kgx materialises the masked messages per input edge
    and reduces them by edge; output and d/dx equal the oracle's with the same mask."""
    from keras_geometric_amd.layers import SAGEConv

    N, F, Fo, E, p = 900, 24, 16, 9000, 0.25
    s, d = rmat_edges(41, scale_for(N), N, 0, E)
    ei = np.stack([s, d]).astype(np.int32)
    x = np.random.default_rng(1).standard_normal((N, F)).astype(np.float32)
    kw = {"pool_hidden_dim": 20} if aggregator == "pooling" else {}
    layer = SAGEConv(Fo, aggregator=aggregator, dropout_rate=p, **kw)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    w = [T(np.asarray(a)) for a in layer.get_weights()]
    torch.manual_seed(321)
    seed = int(torch.randint(0, 2**62, (1,)).item())  # the draw the layer makes
    torch.manual_seed(321)
    y = layer([xd, T(ei).to(dev)], training=True)
    gout = np.random.default_rng(2).standard_normal((N, Fo)).astype(np.float32)
    y.backward(T(gout).to(dev))
    mask = kops.dropout_mask(seed, p, torch.arange(E, dtype=torch.int32, device=dev), F).cpu()
    xr = T(x).requires_grad_(True)
    if aggregator == "pooling":  # Layer.weights order: bias, pool kernel, pool bias, lin_neigh, lin_self
        yr = R.sage_forward(xr, T(ei), w[3], w[4], w[0], "pooling", pool=(w[1], w[2], "relu"), msg_mask=mask)
    else:  # bias, lin_neigh, lin_self
        yr = R.sage_forward(xr, T(ei), w[1], w[2], w[0], aggregator, msg_mask=mask)
    yr.backward(T(gout))
    assert rel(y, yr) <= 1e-5
    # d/dx sums dOut W^T products over each node's out-edges plus the root term,
    # GEMM and sum orders differing from the CPU's: bound 3e-5 (sum measured 1.1e-5)
    assert rel(xd.grad, xr.grad) <= 3e-5
    y_inf = layer([xd, T(ei).to(dev)], training=False)  # inference ignores the rate
    y_ref = R.sage_forward(T(x), T(ei), *(([w[3], w[4], w[0], "pooling"]) if aggregator == "pooling"
                                          else [w[1], w[2], w[0], aggregator]),
                           **({"pool": (w[1], w[2], "relu")} if aggregator == "pooling" else {}))
    assert rel(y_inf, y_ref) <= 1e-5
