"""float64 restatement of the fused aggregate -> transform for the GPU parity
tests (test infrastructure, imported by tests only).

    y[i] = b + PRE( REDUCE_{e in CSR row i} x[col_e] * w_e ) @ W

REDUCE follows the reference aggregators (aggregators.py:48-232): sum, mean =
sum / max(count, 1e-8) with the count in fp32, max / min with the isinf guard
(a row with no message, or an infinite extreme, gives 0); the message is the
fp32 product x_j * w_e, as GCNConv.message computes it (gcn_conv.py:233-248);
PRE is GIN's (1+eps) x_i + aggr (gin_conv.py:216-222).  Sums and the product
with W run in float64 on the device, over the whole graph in row chunks, so a
full-size launch is checked on every row, not a sample.

`check` compares a kernel's output with it under the forward-error bound of
the fp32 computation, |y - ref| <= tol * max(1, |aggr|_abs @ |W| + |b|)
(|aggr|_abs: the same reduction over |messages| for sum / mean, |aggr| for
max / min), and on a failure names the row, the feature and the kernel that
owns the row in the schedule (main / hub-split + fix-up / short / tiny),
so a HIP-vs-HIP mismatch says which side is wrong.
"""

from __future__ import annotations

import torch

RED = {"sum": 0, "mean": 1, "max": 2, "min": 3}


def reference(g, x, W, red: str, weighted: bool, bias=None, pre_gin: bool = False, gin_scale: float = 1.0,
              chunk_edges: int = 1 << 23):
    """(y, scale): float64 [n, F_out] each."""
    dev = x.device
    n, F = g.n_dst, x.shape[1]
    rowptr = g.rowptr.long()
    col = g.col.long()
    w = g.w if weighted else None
    W64 = W.double()
    y = torch.empty((n, W.shape[1]), dtype=torch.float64, device=dev)
    scale = torch.empty_like(y)
    b64 = bias.double() if bias is not None else torch.zeros(W.shape[1], dtype=torch.float64, device=dev)
    r0 = 0
    while r0 < n:
        target = rowptr[r0] + chunk_edges
        r1 = int(torch.searchsorted(rowptr, target, right=True)) - 1
        r1 = min(max(r1, r0 + 1), n)
        e0, e1 = int(rowptr[r0]), int(rowptr[r1])
        deg = rowptr[r0 + 1: r1 + 1] - rowptr[r0: r1]
        seg = torch.repeat_interleave(torch.arange(r1 - r0, device=dev), deg, output_size=e1 - e0)
        m = x[col[e0:e1]]
        if w is not None:
            m = m * w[e0:e1, None]  # fp32 products, as the kernels (__fmul_rn)
        if red in ("sum", "mean"):
            a = torch.zeros((r1 - r0, F), dtype=torch.float64, device=dev).index_add_(0, seg, m.double())
            aa = torch.zeros_like(a).index_add_(0, seg, m.double().abs())
            if red == "mean":
                cnt = deg.to(torch.float32).clamp_min(1e-8).double()[:, None]
                a, aa = a / cnt, aa / cnt
        else:
            op = "amax" if red == "max" else "amin"
            init = float("-inf") if red == "max" else float("inf")
            a32 = torch.full((r1 - r0, F), init, dtype=torch.float32, device=dev)
            a32.scatter_reduce_(0, seg[:, None].expand(-1, F), m, op, include_self=True)
            a32 = torch.where(torch.isinf(a32), torch.zeros_like(a32), a32)
            a = a32.double()
            aa = a.abs()
        if pre_gin:
            xr = x[r0:r1].double()
            a = gin_scale * xr + a
            aa = abs(gin_scale) * xr.abs() + aa
        y[r0:r1] = a @ W64 + b64
        scale[r0:r1] = aa @ W64.abs() + b64.abs()
        r0 = r1
    return y, scale


def owners(g, rows: torch.Tensor) -> list:
    """Which kernel reduced each row: 'split' (hub chunks + fix-up), 'main',
    'short' (degree <= 7 suffix) or 'tiny' (degree <= 2 records), per the
    graph's schedule and tiny-row records as the last launch used them."""
    items = g.items
    if items is None:
        return ["rows"] * rows.numel()
    n_items = items.shape[0]
    pos = torch.full((g.n_dst,), -1, dtype=torch.long, device=items.device)
    pos[items[:, 0].long()] = torch.arange(n_items, device=items.device)
    tiny = getattr(g, "_kgx_tiny", None)
    tiny_start = tiny[2] if tiny and tiny[0] is not None else n_items
    n_long = g.n_long if g.n_long >= 0 else n_items
    out = []
    for r in rows.tolist():
        p = int(pos[r])
        if p < 0:
            out.append("none")
        elif int(items[p, 3]) >= 0:
            out.append("split")
        elif p < n_long:
            out.append("main")
        elif p < tiny_start:
            out.append("short")
        else:
            out.append("tiny")
    return out


def check(y, g, ref, label: str = "", tol: float = 1e-5) -> float:
    """Assert y (fp32 kernel output) within tol of ref = reference(...); returns
    the max scaled error.  On failure the message names the worst rows, their
    features and owning kernels."""
    y64, scale = ref
    err = (y.double() - y64).abs() / scale.clamp_min(1.0)
    mx = float(err.max())
    if not mx <= tol:  # NaN fails too
        bad_rows = torch.nonzero((err > tol).any(1)).flatten()
        worst = torch.argsort(err.max(1).values, descending=True)[:8]
        own = owners(g, worst)
        lines = []
        for r, o in zip(worst.tolist(), own):
            f = int(err[r].argmax())
            lines.append(f"row {r} ({o} kernel) feature {f}: got {float(y[r, f]):.7g} "
                         f"ref {float(y64[r, f]):.7g} scaled err {float(err[r, f]):.3g}")
        raise AssertionError(f"{label}: {bad_rows.numel()} rows beyond {tol} (max {mx:.3g}); worst:\n  "
                             + "\n  ".join(lines))
    return mx
