"""Known-answer tests of the oracle's outflow boundary-face terms
(do_vmult_boundary operator_ns.cc:1195-1295, effective_beta_face :423-457),
on the cylinder decks' outflow boundary (id 1, the plane x = L) with no
constraints, so that every face contribution is visible:

  * Nitsche, u = e_0 constant: the face part of vmult sums to
    sum_F beta_F |F| over the x-velocity dofs (grad u = 0, the test
    functions' normal derivatives sum to 0, the basis is a partition of 1);
  * Nitsche, u_0 = x: sum_F (beta_F L - nu) |F|;
  * cut with u* . n > 0 (outflow): no face term; u* = -e_0: -sum_F beta_F |F|;
  * Nitsche residual: R(u) - R(0) = -(face part of vmult)(u), R(0) carries
    the target: sum_F beta_F |F| for g = e_0;
  * the element matrices (orc_cell_matrix, faces included) assemble to the
    operator: A x == vmult(x), diag(A) == the diagonal.
parity unpinned w.r.t. the reference binary (no golden data), as the oracle."""
import numpy as np
import pytest
import scipy.sparse as sp

import glsmesh as gm
import oracle as orc
from helpers import Case, deck, rel_err

DECKS2 = [("input_turek_2D_Re20_stat.json", 0), ("input_hoffmann_3D_Re3900.json", 0)]


def _setup(name, n_ref, kind, u_lin, nu=None):
    d = deck(name)
    m = d.mesh(n_ref)
    cmask = np.zeros(m.n_nodes, dtype=np.uint8)
    params, w = d.operator_parameters(2.5e-4)
    if nu is not None:
        params["nu"] = nu
    case = Case(m, cmask, params, w, u_inf=d.u_max)
    cells, fno = gm.boundary_faces(m, 1)
    ops = []
    for faces in (True, False):
        om = orc.OracleMesh(m, cmask)
        o = orc.Oracle(om, **params)
        o._om = om
        if faces:
            o.set_outflow_faces(cells, fno, kind)
        o.set_linearization_point(u_lin)
        if params["order"] > 0:
            o.set_previous_solution(case.hist, w)
        ops.append(o)
    return m, case, ops[0], ops[1], cells, fno, params


def _face_area_beta(m, cells, fno):
    """sum_F beta_F |F| from the face nodes' extents (the outflow faces are
    axis-aligned rectangles / segments in the plane x = L)."""
    n, k, dim = m.degree + 1, m.degree, m.dim
    meas, _ = m.cell_measure()
    p = np.arange(n ** dim)
    ia = [p % n, (p // n) % n, p // (n * n)]
    tot = 0.0
    for c, f in zip(cells, fno):
        a, side = f // 2, f % 2
        X = m.coords[np.asarray(m.cell_nodes[c])[ia[a] == side * k]]
        ext = X.max(axis=0) - X.min(axis=0)
        area = np.prod([ext[e] for e in range(dim) if e != a])
        h = (np.sqrt(4 * meas[c] / np.pi) if dim == 2 else (6 * meas[c] / np.pi) ** (1 / 3)) / k
        tot += area / h ** (k + 1)
    return tot


def _const(m, comp, val):
    v = np.zeros(m.n_dofs)
    v[comp::m.dim + 1] = val
    return v


@pytest.mark.parametrize("name,n_ref", DECKS2)
def test_faces_found(name, n_ref):
    m = deck(name).mesh(n_ref)
    cells, fno = gm.boundary_faces(m, 1)
    assert len(cells) > 0 and np.all(fno == 1)  # x+ faces
    L = m.coords[:, 0].max()
    om = orc.OracleMesh(m, np.zeros(m.n_nodes, dtype=np.uint8))
    params, _ = deck(name).operator_parameters()
    o = orc.Oracle(om, **params)
    o.set_outflow_faces(cells, fno, "nitsche")
    x = o.outflow_face_points()
    assert np.allclose(x[..., 0], L)


@pytest.mark.parametrize("name,n_ref", DECKS2)
def test_nitsche_constant_and_linear(name, n_ref):
    d = deck(name)
    m0 = d.mesh(n_ref)
    u_lin = _const(m0, 0, 1.0)
    m, case, of, o0, cells, fno, params = _setup(name, n_ref, "nitsche", u_lin)
    ab = _face_area_beta(m, cells, fno)
    u = _const(m, 0, 1.0)
    dv = of.vmult(u) - o0.vmult(u)
    assert abs(dv[0::m.dim + 1].sum() - ab) < 1e-9 * ab
    assert np.abs(dv[m.dim::m.dim + 1]).max() == 0.0  # no pressure face term
    u = np.zeros(m.n_dofs)
    u[0::m.dim + 1] = m.coords[:, 0]
    L = m.coords[:, 0].max()
    dv = of.vmult(u) - o0.vmult(u)
    # sum_F (beta_F L - nu) |F|: nu sum_F |F| = nu * (outflow area)
    H = m.params["height"]
    out_area = H if m.dim == 2 else H * H
    assert abs(dv[0::m.dim + 1].sum() - (L * ab - params["nu"] * out_area)) < 1e-9 * L * ab


@pytest.mark.parametrize("name,n_ref", DECKS2)
def test_cut_sign(name, n_ref):
    d = deck(name)
    m0 = d.mesh(n_ref)
    u = _const(m0, 0, 1.0)
    # outflow through x = L: min(0, u* . n) = 0, no face term
    m, _, of, o0, cells, fno, _ = _setup(name, n_ref, "cut", _const(m0, 0, 1.0))
    assert np.abs(of.vmult(u) - o0.vmult(u)).max() < 1e-12 * (1 + np.abs(o0.vmult(u)).max())
    # backflow u* = -e_0: -beta_F |F|
    m, _, of, o0, cells, fno, _ = _setup(name, n_ref, "cut", _const(m0, 0, -1.0))
    ab = _face_area_beta(m, cells, fno)
    dv = of.vmult(u) - o0.vmult(u)
    assert abs(dv[0::m.dim + 1].sum() + ab) < 1e-9 * ab
    # residual: u* is the current value -e_0, the face term beta (-1)(-1) v,
    # negated by evaluate_residual
    dr = of.evaluate_residual(-u) - o0.evaluate_residual(-u)
    assert abs(dr[0::m.dim + 1].sum() + ab) < 1e-9 * ab


@pytest.mark.parametrize("name,n_ref", DECKS2)
def test_nitsche_residual(name, n_ref):
    d = deck(name)
    m0 = d.mesh(n_ref)
    m, case, of, o0, cells, fno, _ = _setup(name, n_ref, "nitsche", _const(m0, 0, 1.0))
    g = np.zeros((len(cells), (m.degree + 1) ** (m.dim - 1), m.dim))
    g[..., 0] = 1.0
    of.set_outflow_target(g)
    ab = _face_area_beta(m, cells, fno)
    zero = np.zeros(m.n_dofs)
    r0 = of.evaluate_residual(zero) - o0.evaluate_residual(zero)
    assert abs(r0[0::m.dim + 1].sum() - ab) < 1e-9 * ab
    u = case.src
    ru = of.evaluate_residual(u) - o0.evaluate_residual(u)
    dv = of.vmult(u) - o0.vmult(u)
    assert rel_err(ru - r0, -dv) < 1e-10


@pytest.mark.parametrize("name,n_ref", DECKS2)
@pytest.mark.parametrize("kind", ["cut", "nitsche"])
def test_cell_matrix_assembles(name, n_ref, kind):
    d = deck(name)
    m0 = d.mesh(n_ref)
    rng = np.random.default_rng(5)
    u_lin = _const(m0, 0, -1.0) + 0.1 * rng.standard_normal(m0.n_dofs)
    m, case, of, _, cells, fno, _ = _setup(name, n_ref, kind, u_lin)
    nc, nq = m.dim + 1, (m.degree + 1) ** m.dim
    cn = np.asarray(m.cell_nodes, dtype=np.int64)
    rows, cols, vals = [], [], []
    for c in range(m.n_cells):
        E = of.cell_matrix(c)
        dofs = (cn[c][:, None] * nc + np.arange(nc)[None, :]).ravel()
        rows.append(np.repeat(dofs, len(dofs)))
        cols.append(np.tile(dofs, len(dofs)))
        vals.append(E.ravel())
    A = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(m.n_dofs, m.n_dofs))
    x = case.src
    assert rel_err(A @ x, of.vmult(x)) < 1e-12
    assert rel_err(A.diagonal(), of.diagonal()) < 1e-12
