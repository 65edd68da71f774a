"""Where GPUTEST_r04's wrong row ran (a CPU reconstruction, no GPU).

tests/test_gpu_tiny.py::test_tiny_tail_bit_identical[True-min] failed once in
round 4: 128 of 7,680,000 elements differed, all in row 29312 (largest error
0.0216 at column 55).  This rebuilds that test's graph (R-MAT seed 5,
60,000 nodes, 240,000 edges, + self loops) with the bit-exact restatement
oracle/rmat.py, then the degree-descending schedule kgx_schedule_build emits
(graph_build.hip: exact degree, ties by row id; rows of degree >= split_len
cut into chunks) and spmm_gemm_kernel's launch (kgx_spmm_gemm: grid =
min(ceil(n_long / 16), resident slots); block b takes 16-item tiles b, b +
grid, ...), and prints the tile that reduced row 29312, the degrees of its 16
rows and of the block's next tile.

    python tools/r4_wrong_row.py [row]
"""

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import rmat  # noqa: E402

N, E, SEED = 60_000, 240_000, 5
GROUPS = 16
RESIDENT = 2 * 256  # spmm_gemm_kernel: 4 waves / SIMD at <= 128 VGPRs -> 2 blocks per CU, 256 CUs


def main(row: int = 29312) -> None:
    s, d = rmat.rmat_edges(SEED, rmat.scale_for(N), N, 0, E)
    deg = np.bincount(d, minlength=N) + 1  # + the self loop
    # graph.default_split_len at F 128: a quarter of a group's share, pow2 in [256, 8192]
    share = max(1, int(deg.sum()) // (2048 * 256 // 32))
    split_len = int(min(8192, max(256, 1 << (max(share // 4, 1).bit_length() - 1))))
    order = np.lexsort((np.arange(N), -np.minimum(deg, (1 << 24) - 1)))
    items = []
    for r in order:
        if deg[r] >= split_len:
            nc = (deg[r] + split_len - 1) // split_len
            items += [(r, c * split_len, min(deg[r], (c + 1) * split_len), c) for c in range(nc)]
        else:
            items.append((r, 0, deg[r], -1))
    items = np.array(items)
    ideg = items[:, 2] - items[:, 1]
    short = (ideg <= 7) & (items[:, 3] < 0)
    n_long = int(np.nonzero(~short)[0][-1]) + 1
    grid = min((n_long + GROUPS - 1) // GROUPS, RESIDENT)
    p = int(np.nonzero(items[:, 0] == row)[0][0])
    tile = p // GROUPS
    print(f"row {row}: in-degree {deg[row]} (with its self loop); split_len {split_len}; "
          f"items {len(items)}, main-kernel items n_long {n_long}, grid {grid} blocks")
    print(f"item {p}: tile {tile} -> block {tile % grid}, iteration {tile // grid}, row group {p % GROUPS} "
          f"(wave {p % GROUPS // 2}, which it shares with group {(p % GROUPS) ^ 1})")
    base = tile * GROUPS
    print("tile rows (row, degree):", [(int(items[base + j, 0]), int(ideg[base + j])) for j in range(GROUPS)])
    nxt = base + grid * GROUPS
    print("the block's next tile:", "none (past n_long: every group's prefetch has pn = 0)" if nxt >= n_long
          else [int(ideg[nxt + j]) if nxt + j < n_long else None for j in range(GROUPS)])


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 29312)
