"""The multigrid restatement's coarse direct solve (tests/mg_ref.py,
TEST INFRASTRUCTURE): the coarse matrix assembled from the oracle's element
matrices equals the matrix of the oracle's vmult (columns of unit-vector
applies: identity rows and columns on the constrained dofs), and the
free-block LU solve equals the dense solve of that matrix."""
import numpy as np
import pytest

import glsinputs as gi
from helpers import deck
from mg_ref import OracleGMG


@pytest.mark.parametrize("name", ["input_turek_2D_Re20_stat.json", "input_turek_2D_Re100.json"])
def test_coarse_matrix_from_element_matrices(name):
    d = deck(name)
    meshes = [d.mesh(0), d.mesh(1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=-1)
    A = ref.coarse_matrix()
    n = meshes[0].n_dofs
    cols = np.empty((n, n))
    e = np.zeros(n)
    for j in range(n):
        e[j] = 1.0
        cols[:, j] = ref.ops[0].vmult(e)
        e[j] = 0.0
    assert np.abs(A - cols).max() <= 1e-12 * np.abs(cols).max()
    b = gi.rnd(5, n)
    x = ref.coarse_direct(b)
    assert np.linalg.norm(x - np.linalg.solve(cols, b)) <= 1e-10 * np.linalg.norm(x)
