"""numpy restatement of kgx_rmat_edges (keras-geometric_amd/csrc/graph_build.hip).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Counter-based R-MAT: edge k, level l draws r = splitmix64(splitmix64(seed) +
64*k + l) >> 40 (24 bits) and picks quadrant a / b / c / d by integer
thresholds; ids are taken mod n and relabelled by a 4-round keyed Feistel
permutation on 2*ceil(scale/2) bits with cycle walking.  All arithmetic is
uint64 modulo 2^64, so this restatement and the GPU kernel agree bit for bit.
"""

from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def prob24(p: float) -> int:
    return int(round(p * (1 << 24)))


def _feistel(x, keys, hb):
    mask = np.uint64((1 << hb) - 1)
    L = x >> np.uint64(hb)
    R = x & mask
    for k in keys:
        nl = R
        R = L ^ (splitmix64(np.uint64(k) ^ R) & mask)
        L = nl
    return (L << np.uint64(hb)) | R


def relabel(x, seed: int, scale: int, n: int):
    hb = (scale + 1) // 2
    keys = [int(splitmix64(np.uint64(seed) ^ np.uint64((0xA5A5A5A5A5A5A5A5 + i) & 0xFFFFFFFFFFFFFFFF)))
            for i in range(4)]
    y = _feistel(np.asarray(x, dtype=np.uint64), keys, hb)
    bad = y >= np.uint64(n)
    while bad.any():
        y[bad] = _feistel(y[bad], keys, hb)
        bad = y >= np.uint64(n)
    return y


def rmat_edges(seed: int, scale: int, n: int, e_begin: int, e_count: int,
               a: float = 0.57, b: float = 0.19, c: float = 0.19):
    ta = prob24(a)
    tab = ta + prob24(b)
    tabc = tab + prob24(c)
    base = splitmix64(np.uint64(seed))
    k = np.arange(e_begin, e_begin + e_count, dtype=np.uint64)
    s = np.zeros(e_count, dtype=np.uint64)
    d = np.zeros(e_count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for level in range(scale):
            r = (splitmix64(base + k * np.uint64(64) + np.uint64(level)) >> np.uint64(40)).astype(np.uint32)
            sb = (r >= tab).astype(np.uint64)
            db = (((r >= ta) & (r < tab)) | (r >= tabc)).astype(np.uint64)
            s = (s << np.uint64(1)) | sb
            d = (d << np.uint64(1)) | db
    s = relabel(s % np.uint64(n), seed, scale, n)
    d = relabel(d % np.uint64(n), seed, scale, n)
    return s.astype(np.int32), d.astype(np.int32)


def scale_for(n: int) -> int:
    return max(1, int(np.ceil(np.log2(max(n, 2)))))
