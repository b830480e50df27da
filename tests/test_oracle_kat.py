"""Known-answer tests pinning the CPU oracle.

The reference ships no golden data and cannot be built here (deal.II +
p4est + Trilinos absent), so these identities — each a consequence of the
reference's own formulation (operator_ns.cc:919-1182) — are what pins the
oracle: "parity unpinned" against the reference binary itself.
"""
import numpy as np
import pytest

import glsinputs as gi
import glsmesh as gm
import oracle as orc


def _op(mesh, cmask=None, **kw):
    cmask = np.zeros(mesh.n_nodes, np.uint8) if cmask is None else cmask
    om = orc.OracleMesh(mesh, cmask)
    prm = dict(nu=0.01, c1=2.0, c2=1.0, theta=1.0, w0=150.0, dt=0.01, order=2,
               consider_time_derivative=True, increment_form=True,
               cell_wise_stabilization=False)
    prm.update(kw)
    return orc.Oracle(om, **prm), om


def _const_field(mesh, vals):
    nc = mesh.dim + 1
    v = np.zeros(mesh.n_dofs)
    for c in range(nc):
        v[c::nc] = vals[c]
    return v


MESHES = [lambda: gm.hypercube(3, 2, 1), lambda: gm.hypercube(2, 3, 1),
          lambda: gm.cylinder(2, 2, 1), lambda: gm.cylinder(3, 2, 0), lambda: gm.cylinder(3, 1, 1)]


@pytest.mark.parametrize("mk", MESHES)
@pytest.mark.parametrize("increment_form", [True, False])
def test_kat1_partition_of_unity(mk, increment_form):
    mesh = mk()
    dim = mesh.dim
    op, _ = _op(mesh, increment_form=increment_form)
    U = _const_field(mesh, [1.3, -0.4, 0.7][:dim] + [2.0])
    op.set_linearization_point(U)
    op.set_previous_solution([U, np.zeros_like(U), np.zeros_like(U)], [150.0, 0.0, 0.0])
    cvec = [0.3, 0.8, -0.5][:dim] + [0.0]
    dst = op.vmult(_const_field(mesh, cvec))
    vol = op.geometry()[:, :, 0].sum()
    nc = dim + 1
    for c in range(dim):
        assert abs(dst[c::nc].sum() - 150.0 * cvec[c] * vol) < 1e-11 * max(1, abs(150 * vol))
    assert abs(dst[dim::nc].sum()) < 1e-12


@pytest.mark.parametrize("dim,k", [(2, 1), (2, 2), (3, 1), (3, 2), (3, 3)])
def test_kat2_polynomial_exactness(dim, k):
    """Linear trial and linearisation fields on an affine mesh: the sum of all
    test-function rows equals the quadrature of the analytic value term."""
    mesh = gm.hypercube(dim, k, 1)
    nc = dim + 1
    rng = np.random.default_rng(7)
    A, B = rng.normal(size=(dim, dim)), rng.normal(size=(dim, dim))
    U0, u0 = rng.normal(size=dim), rng.normal(size=dim)
    g, h = rng.normal(size=dim), rng.normal(size=dim)
    X = mesh.coords
    lin = np.zeros(mesh.n_dofs)
    src = np.zeros(mesh.n_dofs)
    for d in range(dim):
        lin[d::nc] = U0[d] + X @ A[d]
        src[d::nc] = u0[d] + X @ B[d]
    lin[dim::nc] = 0.3 + X @ g
    src[dim::nc] = -0.2 + X @ h
    w0 = 7.0
    op, _ = _op(mesh, w0=w0, order=0, consider_time_derivative=False)
    op.set_linearization_point(lin)
    dst = op.vmult(src)
    # quadrature points of each cell (affine cells of side 1/2)
    b = np.polynomial.legendre.leggauss(k + 1)
    qp = 0.5 * (b[0] + 1.0)
    geo = op.geometry()
    lo = np.array([X[mesh.cell_nodes[c]].min(axis=0) for c in range(mesh.n_cells)])
    grids = np.meshgrid(*([qp] * dim), indexing="ij")
    pts_ref = np.stack([gg.transpose().ravel() for gg in grids], axis=1)  # x fastest
    tot = np.zeros(nc)
    for c in range(mesh.n_cells):
        xq = lo[c] + 0.5 * pts_ref
        Uq = U0 + xq @ A.T
        uq = u0 + xq @ B.T
        V = w0 * uq + Uq @ B.T + uq @ A.T  # w0 u + (grad u) U + (grad U) u
        jxw = geo[c, :, 0]
        tot[:dim] += jxw @ V
        tot[dim] += jxw.sum() * np.trace(B)
    for c in range(nc):
        assert abs(dst[c::nc].sum() - tot[c]) < 1e-10 * max(1, abs(tot).max())


def _assemble(op, mesh, cmask):
    nc = mesh.dim + 1
    n = mesh.n_dofs
    A = np.zeros((n, n))
    for c in range(mesh.n_cells):
        Ae = op.cell_matrix(c)
        idx = (mesh.cell_nodes[c][:, None] * nc + np.arange(nc)[None, :]).ravel()
        A[np.ix_(idx, idx)] += Ae
    con = np.zeros(n, bool)
    for comp in range(nc):
        con[comp::nc] = (cmask >> comp) & 1
    A[con, :] = 0
    A[:, con] = 0
    A[con, con] = 1.0
    return A


@pytest.mark.parametrize("mk", [lambda: gm.cylinder(2, 2, 0), lambda: gm.cylinder(3, 1, 0)])
@pytest.mark.parametrize("increment_form", [True, False])
def test_kat3_matrix_consistency(mk, increment_form):
    mesh = mk()
    d = gm.read_deck(gm.DECK_DIR + "/input_hoffmann_3D_Re3900.json")
    vel, p, slip = [0, 2], [1], [3, 4, 5, 6]
    cmask = mesh.constraint_mask(vel, p, slip)
    op, _ = _op(mesh, cmask, increment_form=increment_form)
    u = gi.linearization_point(mesh.n_nodes, mesh.dim, 2.0)
    op.set_linearization_point(u)
    op.set_previous_solution(gi.history(u, 2), [150.0, -200.0, 50.0])
    A = _assemble(op, mesh, cmask)
    x = gi.src_vector(mesh.n_dofs)
    assert np.allclose(A @ x, op.vmult(x), rtol=0, atol=1e-11 * np.abs(A @ x).max())
    inv = op.inverse_diagonal()
    dg = np.diag(A)
    ref = np.where(np.abs(dg) > 1e-10, 1.0 / np.where(dg == 0, 1, dg), 1.0)
    assert np.allclose(inv, ref, rtol=1e-12, atol=0)
    del d


@pytest.mark.parametrize("dim", [2, 3])
def test_kat5_symmetry(dim):
    mesh = gm.cylinder(dim, 2, 0) if dim == 2 else gm.hypercube(3, 2, 1)
    op, _ = _op(mesh)
    op.set_linearization_point(np.zeros(mesh.n_dofs))
    op.set_previous_solution([np.zeros(mesh.n_dofs)] * 3, [150.0, 0.0, 0.0])
    nc = dim + 1
    for c in range(min(mesh.n_cells, 4)):
        Ae = op.cell_matrix(c)
        vel = np.array([i for i in range(Ae.shape[0]) if i % nc < dim])
        Avv = Ae[np.ix_(vel, vel)]
        assert np.allclose(Avv, Avv.T, atol=1e-12 * np.abs(Avv).max())


@pytest.mark.parametrize("dim,k", [(2, 1), (2, 2), (3, 1), (3, 2)])
def test_kat6_transfer(dim, k):
    cm, fm = gm.hypercube(dim, k, 1), gm.hypercube(dim, k, 2)
    lat = cm.child_lattice(fm)
    nc = dim + 1
    z = lambda m: np.zeros(m.n_nodes, np.uint8)  # noqa: E731
    ocm, ofm = orc.OracleMesh(cm, z(cm)), orc.OracleMesh(fm, z(fm))

    def poly(X):
        out = 1.0 + X[:, 0] - 0.5 * X[:, 1]
        if k == 2:
            out += X[:, 0] * X[:, 1] - 0.3 * X[:, 0] ** 2
        return out

    src = np.zeros(cm.n_dofs)
    for c in range(nc):
        src[c::nc] = (c + 1) * poly(cm.coords)
    dst = np.zeros(fm.n_dofs)
    orc.prolongate_add(ocm, ofm, lat, dst, src)
    for c in range(nc):
        assert np.allclose(dst[c::nc], (c + 1) * poly(fm.coords), atol=1e-13)
    # restriction is the transpose of prolongation (with constraints)
    cmask_c = (cm.node_boundary > 0).astype(np.uint8) * 3
    cmask_f = (fm.node_boundary > 0).astype(np.uint8) * 3
    ocm, ofm = orc.OracleMesh(cm, cmask_c), orc.OracleMesh(fm, cmask_f)
    rng = np.random.default_rng(3)
    x, y = rng.normal(size=cm.n_dofs), rng.normal(size=fm.n_dofs)
    Px = np.zeros(fm.n_dofs)
    orc.prolongate_add(ocm, ofm, lat, Px, x)
    Ry = np.zeros(cm.n_dofs)
    orc.restrict_add(ocm, ofm, lat, Ry, y)
    assert abs(Px @ y - x @ Ry) < 1e-12 * abs(Px @ y)
    # interpolate_to_mg: injection of the fine nodal values
    back = np.zeros(cm.n_dofs)
    ofm0 = orc.OracleMesh(fm, z(fm))
    orc.interpolate(orc.OracleMesh(cm, z(cm)), ofm0, lat, back, dst)
    assert np.allclose(back, src, atol=1e-13)


def test_bdf_weights():
    dt = 0.1
    assert np.allclose(orc.bdf_weights(1, [dt]), [1 / dt, -1 / dt])
    assert np.allclose(orc.bdf_weights(2, [dt, dt]), [3 / (2 * dt), -2 / dt, 1 / (2 * dt)])
    assert np.allclose(orc.bdf_weights(3, [dt, dt, dt]),
                       np.array([11 / 6, -3, 3 / 2, -1 / 3]) / dt)
    # first step of a BDF2 integrator: effective order 1 (dt history zero)
    assert np.allclose(orc.bdf_weights(2, [dt, 0.0]), [1 / dt, -1 / dt, 0])
    # variable step: weights reproduce derivatives of quadratics exactly
    dts = [0.1, 0.15, 0.07]
    w = orc.bdf_weights(3, dts)
    t = np.array([0.0, -dts[0], -dts[0] - dts[1], -sum(dts)])
    for f, df in [(lambda s: s, 1.0), (lambda s: s ** 2, 0.0), (lambda s: s ** 3, 0.0)]:
        assert abs(w @ f(t) - df) < 1e-9
    # the deck helper agrees with the oracle
    d = gm.read_deck(gm.DECK_DIR + "/input_hoffmann_3D_Re3900.json")
    theta, wd, order, cdt = d.time_integrator(2.5e-4)
    assert order == 2 and theta == 1.0 and cdt == 2.5e-4
    assert np.allclose(wd, orc.bdf_weights(2, [2.5e-4, 2.5e-4]))


def test_penalty_parameters():
    """delta formulas (operator_ns.cc:394-420, :369-388) at a uniform
    velocity on the unit hyper cube."""
    mesh = gm.hypercube(3, 2, 1)
    op, _ = _op(mesh, nu=0.01, dt=0.01)
    U = _const_field(mesh, [3.0, 4.0, 0.0, 0.0])
    op.set_linearization_point(U)
    t, cw = op.tables()
    h = (6 * 0.125 / np.pi) ** (1 / 3) / 2
    u2 = 25.0 + 1e-12
    d1 = 1 / np.sqrt(100.0 ** 2 + 4 * u2 / h ** 2 + 9 * (4 * 0.01 / h ** 2) ** 2)
    assert np.allclose(t[:, :, 0], d1, rtol=1e-13)
    assert np.allclose(t[:, :, 1], np.sqrt(u2) * h / 2, rtol=1e-13)
    hmin = 0.5
    assert np.allclose(cw[:, 0], 2.0 / np.sqrt(100.0 ** 2 + 25.0 / hmin ** 2), rtol=1e-13)
    assert np.allclose(cw[:, 1], 1.0 * hmin, rtol=1e-13)
