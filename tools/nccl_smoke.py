"""RCCL smoke test of the sharded path on a one-GPU box (a measurement helper).

  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/nccl_smoke.py

One rank cannot exercise a real halo, but it runs the product's RCCL plumbing
on the hardware: the "nccl" process group with high-priority streams (as
bench.py creates it), TorchComm's all_to_all_single / async all_to_all_start +
wait() on the side stream, the push-pull planning collectives and the
pipelined ShardedGCNConv / ShardedGINConv forwards -- checked against the
single-GPU layers.  Multi-rank exchange is covered by the gloo and threaded-GPU
tests and by the driver's 8-GPU run.
"""

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", device_id=dev, pg_options=opts)
    import keras_geometric_amd as kgx
    from keras_geometric_amd import distributed as kd
    from keras_geometric_amd import synthetic

    n, e = 200_000, 2_000_000
    comm = kd.TorchComm()
    # async all-to-all through the comm, waited on another stream
    x = torch.arange(1024, dtype=torch.float32, device=dev).view(256, 4)
    out = torch.empty_like(x)
    side = torch.cuda.Stream(priority=-1)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        w = comm.all_to_all_start(out, x, [256], [256])
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(out, x)

    sg = kd.ShardedGraph.rmat(n, e, seed=3, device=dev, comm=comm, n_features=128)
    xs = torch.randn(sg.n_local, 128, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    layer = kd.ShardedGCNConv(128, sg)
    with torch.no_grad():
        y = layer(xs)
    ei = synthetic.rmat_edge_index(n, e, seed=3, device=dev)
    ref_layer = kgx.GCNConv(128)
    with torch.no_grad():
        ref_layer([xs, ei])
        ref_layer.set_weights(layer.get_weights())
        ref = ref_layer([xs, ei])
    err = ((y - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert err <= 1e-5, err

    gsg = kd.ShardedGraph.rmat(n, e, seed=3, device=dev, comm=comm, n_features=128, self_loops=False,
                               gcn_norm=False)
    gin = kd.ShardedGINConv(64, gsg, aggregator="sum", eps_init=0.25)
    with torch.no_grad():
        h = gin(xs)
    ref_gin = kgx.GINConv(64, aggregator="sum", eps_init=0.25)
    with torch.no_grad():
        ref_gin([xs, ei])
        ref_gin.set_weights(gin.conv.get_weights())
        href = ref_gin([xs, ei])
    err2 = ((h - href).abs() / href.abs().clamp_min(1.0)).max().item()
    assert err2 <= 1e-5, err2
    print(f"nccl smoke ok: backend={dist.get_backend()} world={dist.get_world_size()} "
          f"gcn err {err:.2e} gin err {err2:.2e} halo_k={sg.halo_k} pp={sg._pp is not None}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    np.seterr(all="ignore")
    main()
