"""FE_Q_iso_Q1 coarsest multigrid level (main.cc:436-446, "gmg coarse grid
use fe q iso q1" of the sphere and Re20 decks): glsmesh.IsoQ1Mesh runs it as
the Q1 operator on the coarse cells' sub-cells (same support points, QGauss(2)
per sub-cell = QIterated(QGauss(2), k)), and the transfer to the next level
is the Q1 one (the iso-Q1 embedding).

CPU: structure (sub-cell corners are next-level nodes, measures add up), the
oracle transfer's exactness on linear fields through the iso-Q1 level, and the
parent mapping of the sub-cells (main.cc:413-414: the level's MappingQ(k) maps
the iso-Q1 level too): per sub-cell the parent's Q_k map at its Q_k lattice.
GPU: the V-cycle with an iso-Q1 coarse level against the oracle multigrid on
the same levels (the GPU's own omegas / diagonals, as test_gpu_mg.py)."""
import numpy as np
import pytest

import glsinputs as gi
import glsmesh as gm
import oracle as orc
from helpers import deck, rel_err

DECKS = [("input_sphere_amg.json", 1), ("input_turek_2D_Re20_stat.json", 2)]


@pytest.mark.parametrize("name,n_ref", DECKS)
def test_structure(name, n_ref):
    d = deck(name)
    assert d.use_fe_q_iso_q1
    m0, m1 = d.mesh(0), d.mesh(1)
    iso = gm.IsoQ1Mesh(m0)
    assert iso.degree == 1 and iso.n_nodes == m0.n_nodes
    assert iso.n_cells == m0.n_cells * m0.degree ** m0.dim
    ch = iso.child_lattice(m1)
    corners = [0, 2, 6, 8, 18, 20, 24, 26] if m0.dim == 3 else [0, 2, 6, 8]
    assert np.abs(np.asarray(m1.coords)[ch[:, corners]] -
                  np.asarray(m0.coords)[iso.cell_nodes]).max() < 1e-13
    meas, _ = iso.cell_measure()
    assert np.isclose(meas.sum(), m0.cell_measure()[0].sum())


@pytest.mark.parametrize("name,n_ref", DECKS)
def test_iso_transfer_linear_exact(name, n_ref):
    """Prolongation from the iso-Q1 level reproduces a linear field at the
    next level's nodes (multilinear geometry); interpolation back is the
    identity (KAT-6 style)."""
    d = deck(name)
    m0, m1 = d.mesh(0), d.mesh(1)
    iso = gm.IsoQ1Mesh(m0)
    dim, nc = m0.dim, m0.dim + 1
    om0 = orc.OracleMesh(iso, np.zeros(iso.n_nodes, np.uint8))
    om1 = orc.OracleMesh(m1, np.zeros(m1.n_nodes, np.uint8))
    child = iso.child_lattice(m1)
    a = np.array([[0.3, -1.2, 0.7][:dim], [1.1, 0.4, -0.5][:dim], [-0.2, 0.9, 0.6][:dim],
                  [0.5, 0.5, -1.0][:dim]])[:nc]
    f = lambda X: (X @ a.T + np.arange(nc)).ravel()  # noqa: E731
    uc = f(np.asarray(m0.coords))
    uf = np.zeros(m1.n_dofs)
    orc.prolongate_add(om0, om1, child, uf, uc)
    if d.simulation == "sphere":
        # multilinear cells: the reference-space embedding reproduces a
        # physically linear field (on the MappingQ2-curved cylinder cells it
        # reproduces the nodal interpolant in reference coordinates instead)
        assert np.abs(uf - f(np.asarray(m1.coords))).max() < 1e-12
    back = np.zeros(m0.n_dofs)
    orc.interpolate(om0, om1, child, back, uf)
    assert np.abs(back - uc).max() < 1e-12


def _jxw_sum(dim, k, pts):
    """sum of det J w over QGauss(k+1)^dim of the Q_k maps given by their
    (k+1)^dim support points per cell (numpy restatement, independent of the
    oracle and of the library)"""
    n = k + 1
    g = gm._gll_nodes(k)
    x, w = np.polynomial.legendre.leggauss(n)
    x, w = 0.5 * (x + 1), 0.5 * w
    S = np.array([[gm._lagrange(g, i, xq) for i in range(n)] for xq in x])
    D = np.zeros_like(S)
    for i in range(n):  # derivative of the Lagrange basis by the product rule
        for j in range(n):
            if j == i:
                continue
            t = np.ones_like(x) / (g[i] - g[j])
            for m in range(n):
                if m != i and m != j:
                    t = t * (x - g[m]) / (g[i] - g[m])
            D[:, i] += t
    X = pts.reshape((-1,) + (n,) * dim + (dim,))
    if dim == 2:
        jx = np.einsum("qy,px,cyxd->cqpd", S, D, X)
        jy = np.einsum("qy,px,cyxd->cqpd", D, S, X)
        det = jx[..., 0] * jy[..., 1] - jx[..., 1] * jy[..., 0]
        return float(np.einsum("cqp,q,p->", det, w, w))
    jx = np.einsum("rz,qy,px,czyxd->crqpd", S, S, D, X)
    jy = np.einsum("rz,qy,px,czyxd->crqpd", S, D, S, X)
    jz = np.einsum("rz,qy,px,czyxd->crqpd", D, S, S, X)
    det = np.einsum("...i,...i->...", jx, np.cross(jy, jz))
    return float(np.einsum("crqp,r,q,p->", det, w, w, w))


@pytest.mark.parametrize("name,n_ref", DECKS)
def test_mapping_points_parent_map(name, n_ref):
    """The sub-cells' mapping points reproduce the parent MappingQ(k): their
    corners are the sub-cell corner nodes, and the areas / volumes they
    integrate add up to the parent cells' (exact quadrature for the 2D Q2
    map's det J and the sphere's trilinear cells)."""
    d = deck(name)
    m0 = d.mesh(0)
    iso = gm.IsoQ1Mesh(m0)
    k, pts = iso.mapping_points()
    dim, n = m0.dim, k + 1
    assert k == m0.degree and pts.shape == (iso.n_cells, n ** dim, dim)
    corners = [0, n - 1, n * (n - 1), n * n - 1]
    corners = corners + [c + n * n * (n - 1) for c in corners] if dim == 3 else corners
    assert np.abs(pts[:, corners] - np.asarray(m0.coords)[iso.cell_nodes]).max() < 1e-12
    parent = np.asarray(m0.coords)[np.asarray(m0.cell_nodes, dtype=np.int64)]
    vp, vs = _jxw_sum(dim, k, parent), _jxw_sum(dim, k, pts)
    assert abs(vs - vp) < 1e-12 * abs(vp)


class _NoMapping:
    """the iso-Q1 mesh without its parent mapping (multilinear sub-cells)"""

    def __init__(self, iso):
        for a in ("dim", "degree", "n_nodes", "n_cells", "cell_nodes", "coords", "n_dofs"):
            setattr(self, a, getattr(iso, a))
        self.cell_measure = iso.cell_measure


@pytest.mark.parametrize("name,n_ref", DECKS)
def test_oracle_parent_mapping(name, n_ref):
    """Oracle operator on the iso-Q1 level with the parent mapping: the same
    as multilinear sub-cells on the sphere's trilinear cells, different on the
    MappingQ2-curved cylinder cells."""
    d = deck(name)
    m0 = d.mesh(0)
    iso = gm.IsoQ1Mesh(m0)
    vel, p, slip = d.boundary_descriptor()
    cm = iso.constraint_mask(vel, p, slip)
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(m0.n_nodes, m0.dim, d.u_max)
    hist = gi.history(u, params["order"])
    x = gi.rnd(5, iso.n_dofs)
    ys = []
    for mesh in (iso, _NoMapping(iso)):
        o = orc.Oracle(orc.OracleMesh(mesh, cm), **params)
        o.set_linearization_point(u)
        o.set_previous_solution(hist, w)
        ys.append(o.vmult(x))
    diff = rel_err(ys[0], ys[1])
    if d.simulation == "sphere":
        assert diff < 1e-12
    else:
        assert diff > 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_ref,coarse", [("input_sphere_amg.json", 1, 10),
                                               ("input_turek_2D_Re20_stat.json", 2, -1)])
def test_gpu_vcycle_iso_q1(name, n_ref, coarse):
    import torch
    import glsamd
    from mg_ref import OracleGMG
    d = deck(name)
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=coarse, coarse_iso_q1=True)
    assert ops[0].degree == 1 and ops[0].n_cells == meshes[0].n_cells * 2 ** meshes[0].dim
    ref = OracleGMG([gm.IsoQ1Mesh(meshes[0])] + meshes[1:], cm, params, u, hist, w,
                    coarse_iters=coarse)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        if l == 0:
            # the iso-Q1 level's own diagonal (parent mapping on both sides)
            assert rel_err(dl.double().cpu().numpy(), ref.invdiag[0]) < 1e-3
        ref.invdiag[l] = dl.double().cpu().numpy()
    # the level-0 operator itself: FP32 iso-Q1 GPU vs FP64 oracle on the sub-cells
    x0 = gi.rnd(3, meshes[0].n_dofs)
    y0 = ops[0].initialize_dof_vector()
    ops[0].vmult(y0, ops[0]._dev(x0))
    torch.cuda.synchronize()
    assert rel_err(y0.double().cpu().numpy(), ref.ops[0].vmult(x0)) < 2e-5
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    assert rel_err(dst.cpu().numpy(), ref.vcycle(b)) < 5e-4
