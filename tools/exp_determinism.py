"""Run-to-run determinism of the backward paths (a debugging helper).

  python tools/exp_determinism.py

Builds the test graphs of test_gpu_backward.py's GIN-mean and GATv2 cases,
runs forward + backward repeatedly (fresh graph objects and a cleared
allocator cache in between) and reports the largest difference between runs
of the transposed CSR arrays and of the gradients.
"""

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import keras_geometric_amd as kgx  # noqa: E402
from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd.layers import GATv2Conv, GINConv  # noqa: E402
from oracle.rmat import rmat_edges, scale_for  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N = 900
    s, d = rmat_edges(24, scale_for(N), N, 0, 8000)
    ei = torch.from_numpy(np.stack([s, d])).to(dev)
    x0 = torch.from_numpy(np.random.default_rng(25).standard_normal((N, 24)).astype(np.float32)).to(dev)
    gout = torch.from_numpy(np.random.default_rng(26).standard_normal((N, 128)).astype(np.float32)).to(dev)
    ref = {}
    worst = {}
    for it in range(12):
        G.clear_cache() if hasattr(G, "clear_cache") else None
        junk = torch.full((1 << 22,), float("nan"), device=dev)  # dirty the allocator's free blocks
        del junk
        torch.manual_seed(0)
        lay = GATv2Conv(16, heads=8, concat=True, exact=True)
        xd = x0.clone().requires_grad_(True)
        lay([xd, ei])
        with torch.no_grad():
            lay.bias.copy_(torch.linspace(-1, 1, 128, device=dev))
        y = lay([xd, ei])
        y.backward(gout)
        res = {"gat_y": y.detach(), "gat_dx": xd.grad.detach(), "gat_datt": lay.att.grad.detach()}
        torch.manual_seed(0)
        gin = GINConv(32, aggregator="mean")
        xg = x0.clone().requires_grad_(True)
        yg = gin([xg, ei])
        yg.square().sum().backward()
        res["gin_dx"] = xg.grad.detach()
        torch.cuda.synchronize()
        for k, v in res.items():
            if k not in ref:
                ref[k] = v.clone()
            else:
                dd = (v - ref[k]).abs().max().item()
                nan = bool(torch.isnan(v).any())
                worst[k] = max(worst.get(k, 0.0), dd if not nan else float("inf"))
    print({k: f"{v:.3g}" for k, v in worst.items()}, flush=True)


if __name__ == "__main__":
    main()
