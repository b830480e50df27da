"""TEST INFRASTRUCTURE: the tiling check of discovered bricks; the shuffled
mesh itself is glsmesh.ShuffledMesh (bench.py times it too)."""
import numpy as np

from glsmesh import ShuffledMesh  # noqa: F401

def check_tiling(cell_nodes, dim, degree, shape, perm):
    """Every brick of `shape` cells (consecutive in perm) forms one node
    lattice: a node at one lattice position, a position with one node."""
    n, k = degree + 1, degree
    bx, by, bz = shape
    cpb = bx * by * bz
    cn = np.asarray(cell_nodes, dtype=np.int64)
    assert sorted(perm.tolist()) == list(range(len(cn)))
    assert len(cn) % cpb == 0
    Lx, Ly = k * bx + 1, k * by + 1
    p = np.arange(n ** dim)
    i, j, l = p % n, (p // n) % n, (p // (n * n) if dim == 3 else 0 * p)
    for b in range(len(cn) // cpb):
        lat = {}
        for lc in range(cpb):
            cx, cy, cz = lc % bx, (lc // bx) % by, lc // (bx * by)
            li = (cx * k + i) + Lx * ((cy * k + j) + Ly * (cz * k + l))
            for q, node in zip(li, cn[perm[b * cpb + lc]]):
                assert lat.setdefault(int(q), int(node)) == node
        assert len(set(lat.values())) == len(lat)
