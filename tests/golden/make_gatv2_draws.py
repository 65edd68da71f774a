"""Weight draws for the GATv2 backward conditioning tests (tests/test_gatv2_conditioning.py).

    python tests/golden/make_gatv2_draws.py

The graph, features and output gradient are those of
tests/test_gpu_backward.py::test_gatv2_layer_backward (R-MAT seed 24, N=900,
E=8000; x seed 25; grad seed 26; bias seed 27), 8 heads x 16 channels, concat.
The weights are glorot-uniform draws (the layer's initialisers) from torch's
CPU generator with the seeds below, saved as arrays so the test does not
depend on any RNG implementation.

Seeds 10, 57 and 167 are the draws, among CPU seeds 0-199, on which the fp32
oracle's gradients miss the fp64 oracle's by more than 1e-5 (6e-4 - 1.2e-3 in
d/dx, 5e-3 - 1.1e-2 in d/dkernel): in each, exactly one leaky-ReLU input z lies
within 6e-9 - 3.5e-8 of zero and fp32 and fp64 put it on opposite sides, where
the derivative jumps from 1 to 0.2 (tools/exp_gatv2_seeds.py finds the same on
the GPU's own draws: CUDA seeds 25 and 47 of 0-47).  Seed 0 is well
conditioned.  Round 2's unexplained 7.7e-4 miss has this size.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

OUT = Path(__file__).resolve().parent / "gatv2_bwd_draws.npz"
SEEDS = {"well": [0], "kink": [10, 57, 167]}
FI, HEADS, C = 24, 8, 16


def draw(seed: int) -> tuple[np.ndarray, np.ndarray]:
    g = torch.Generator().manual_seed(seed)
    out = HEADS * C
    kern = (torch.rand(FI, out, generator=g) * 2 - 1) * (6.0 / (FI + out)) ** 0.5
    att = (torch.rand(1, HEADS, C, generator=g) * 2 - 1) * (6.0 / (HEADS + C)) ** 0.5
    return kern.numpy(), att.numpy()


def main() -> None:
    arrays = {}
    for kind, seeds in SEEDS.items():
        for s in seeds:
            k, a = draw(s)
            arrays[f"{kind}_{s}_kernel"] = k
            arrays[f"{kind}_{s}_att"] = a
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT} ({', '.join(sorted(arrays))})")


if __name__ == "__main__":
    main()
