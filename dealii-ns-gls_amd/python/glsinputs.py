"""Platform-independent synthetic inputs of SURVEY §8d.

rnd(seed, i) = ((splitmix64(seed * 2^32 + i) >> 11) * 2^-53) * 2 - 1  in [-1, 1)

  src                 = rnd(1, i)
  u* velocity x       = U_inf * (1 + 0.1 rnd(2, i)), y/z = 0.1 U_inf rnd(2, i),
  p*                  = rnd(2, i)
  history[1], [2]     = 0.99 u*, 0.98 u*
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def rnd(seed, n):
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed) * np.uint64(1 << 32) + i
    r = (splitmix64(x) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    return r * 2.0 - 1.0


def src_vector(n_dofs):
    return rnd(1, n_dofs)


def linearization_point(n_nodes, dim, u_inf):
    nc = dim + 1
    r = rnd(2, n_nodes * nc)
    u = np.empty(n_nodes * nc)
    u[0::nc] = u_inf * (1.0 + 0.1 * r[0::nc])
    for d in range(1, dim):
        u[d::nc] = 0.1 * u_inf * r[d::nc]
    u[dim::nc] = r[dim::nc]
    return u


def history(u_star, order):
    """SolutionHistory vectors [0..order] (index 0 = current, unused)."""
    h = [u_star.copy()]
    for i in range(1, order + 1):
        h.append((1.0 - 0.01 * i) * u_star)
    return h
