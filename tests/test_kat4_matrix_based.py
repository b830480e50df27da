"""KAT-4: the reference's second formulation of the same
operator, NavierStokesOperatorMatrixBased::compute_system_matrix_and_vector
(operator_ns.cc:1600-1740), restated here independently of the oracle — an
FEValues-style quadrature loop over dense Q_k shape values and gradients
(no sum factorisation, no tables) — and compared element by element with
the matrix-free fixed-point operator's element matrices (orc_cell_matrix,
the unit-vector applies of MatrixFreeTools::compute_matrix) and, on the GPU,
with gls_op_element_matrices.

Conditions under which the two formulations coincide:
fixed-point branch (increment_form = false), theta scheme with theta = 1
(weights 1/tau), consider_time_derivative = false, cell-wise stabilization,
linearization point = previous solution (delta_1 from the same u_max),
affine cells (the matrix-based FEValues uses the Q1 mapping), no
constraints.  Then MB = diag(tau I_vel, I_p) A_mf, term by term
(velocity a..f :1684-1691 <-> :1019-1044, pressure a, b :1694-1695 <->
:1050-1057; delta :1660-1679 <-> :369-388)."""
import numpy as np
import pytest

import glsinputs as gi
import glsmesh as gm
import oracle as orc
from helpers import rel_err

TAU = 0.01
PRM = dict(nu=0.02, c1=2.0, c2=1.0)


class AffineMesh:
    """A hypercube mesh under the affine map x -> A x + b: parallelogram /
    parallelepiped cells, so that the Q1 and Q_k mappings coincide."""

    def __init__(self, base, A, b):
        self.base = base
        self.dim, self.degree = base.dim, base.degree
        self.n_cells, self.n_nodes = base.n_cells, base.n_nodes
        self.cell_nodes = np.asarray(base.cell_nodes)
        self.coords = np.asarray(base.coords) @ np.asarray(A).T + np.asarray(b)
        self.A = np.asarray(A)

    @property
    def n_dofs(self):
        return self.n_nodes * (self.dim + 1)

    def cell_measure(self):
        meas, _ = self.base.cell_measure()
        meas = meas * abs(np.linalg.det(self.A))
        # cell->minimum_vertex_distance(): the 2^dim corners of the cell
        n, dim = self.degree + 1, self.dim
        corners = [i + n * (j + n * l) for l in ((0, n - 1) if dim == 3 else (0,))
                   for j in (0, n - 1) for i in (0, n - 1)]
        X = self.coords[self.cell_nodes[:, corners]]
        d = np.linalg.norm(X[:, :, None, :] - X[:, None, :, :], axis=-1)
        d[:, np.arange(len(corners)), np.arange(len(corners))] = np.inf
        return meas, d.min(axis=(1, 2))


def _lagrange(nodes, i, x):
    """value and derivative of the 1D Lagrange polynomial i on `nodes`"""
    v, dv = 1.0, 0.0
    for j in range(len(nodes)):
        if j == i:
            continue
        prod = 1.0 / (nodes[i] - nodes[j])
        for m in range(len(nodes)):
            if m != i and m != j:
                prod *= (x - nodes[m]) / (nodes[i] - nodes[m])
        dv += prod
        v *= (x - nodes[j]) / (nodes[i] - nodes[j])
    return v, dv


def _gll(k):
    return {1: [0.0, 1.0], 2: [0.0, 0.5, 1.0],
            3: [0.0, 0.5 - np.sqrt(5) / 10, 0.5 + np.sqrt(5) / 10, 1.0]}[k]


def matrix_based_cell(mesh, c, u_star, u_0):
    """The cell matrix of operator_ns.cc:1627-1695 (FESystem(FE_Q(k), dim+1),
    QGauss(k+1), Q1 mapping), local dof = node * (dim+1) + component."""
    dim, k = mesh.dim, mesh.degree
    n, nc = k + 1, dim + 1
    nq = n ** dim
    nd = nq * nc
    nodes = _gll(k)
    xg, wg = np.polynomial.legendre.leggauss(n)
    xg, wg = 0.5 * (xg + 1), 0.5 * wg
    lat = [(i % n, (i // n) % n, i // (n * n)) for i in range(nq)]
    cn = mesh.cell_nodes[c]
    X = mesh.coords[cn]
    # delta_1, delta_2 (:1660-1679): u_max over the q points of u_0, h the
    # minimum vertex distance
    _, hmin = mesh.cell_measure()
    h = hmin[c]
    phis, grads, jxws = [], [], []
    for q in range(nq):
        xi = [xg[lat[q][d]] for d in range(dim)]
        w = np.prod([wg[lat[q][d]] for d in range(dim)])
        phi = np.ones(nq)
        dphi = np.ones((nq, dim))
        for i in range(nq):
            vals = [_lagrange(nodes, lat[i][d], xi[d]) for d in range(dim)]
            phi[i] = np.prod([v for v, _ in vals])
            for a in range(dim):
                dphi[i, a] = np.prod([vals[d][1] if d == a else vals[d][0] for d in range(dim)])
        J = X.T @ dphi                      # dx_d / dxi_a
        grad = dphi @ np.linalg.inv(J)      # d phi_i / dx_e
        phis.append(phi)
        grads.append(grad)
        jxws.append(abs(np.linalg.det(J)) * w)
    U0 = np.stack([u_0[cn * nc + d] for d in range(dim)], axis=1)
    US = np.stack([u_star[cn * nc + d] for d in range(dim)], axis=1)
    u_max = max(np.linalg.norm(phi @ U0) for phi in phis)
    nu, c1, c2 = PRM["nu"], PRM["c1"], PRM["c2"]
    if nu < h:
        d1 = c1 / np.sqrt(1.0 / TAU ** 2 + u_max ** 2 / h ** 2)
        d2 = c2 * h
    else:
        d1, d2 = c1 * h * h, c2 * h * h
    theta, tau = 1.0, TAU
    E = np.zeros((nd, nd))
    for phi, grad, jxw in zip(phis, grads, jxws):
        us = phi @ US
        # per local dof: velocity value, gradient [d][e], divergence, eps;
        # pressure value and gradient
        V = np.zeros((nd, dim))
        G = np.zeros((nd, dim, dim))
        Pv = np.zeros(nd)
        Pg = np.zeros((nd, dim))
        for i in range(nq):
            for comp in range(nc):
                I = i * nc + comp
                if comp < dim:
                    V[I, comp] = phi[i]
                    G[I, comp, :] = grad[i]
                else:
                    Pv[I] = phi[i]
                    Pg[I] = grad[i]
        div = np.einsum("ndd->n", G)
        eps = 0.5 * (G + G.transpose(0, 2, 1))
        conv = np.einsum("nde,e->nd", G, us)           # grad_u * u_star
        # rows i: test, columns j: trial (:1684-1695)
        lhs = (V @ V.T                                                   # a
               + theta * tau * (V @ conv.T)                              # b: (grad u_j u*) . v_i
               - tau * np.outer(div, Pv)                                 # c: p_j div v_i
               + theta * tau * 2 * nu * np.einsum("ide,jde->ij", eps, eps)   # d
               + theta * tau * d1 * np.einsum("jd,id->ij", conv + Pg, conv)  # e
               + theta * tau * d2 * np.outer(div, div)                   # f
               + theta * np.outer(Pv, div)                               # pressure a
               + d1 * np.einsum("jd,id->ij", Pg + theta * conv, Pg))     # pressure b
        E += jxw * lhs
    return E


CASES = [
    (2, 2, 2, [[1.3, 0.4], [-0.2, 0.9]]),
    (3, 2, 1, [[1.1, 0.3, -0.1], [0.0, 0.8, 0.2], [0.15, -0.1, 1.2]]),
    (2, 3, 1, [[0.7, -0.3], [0.25, 1.1]]),
]


def _setup(dim, k, n_ref, A):
    base = gm.hypercube(dim, k, n_ref)
    mesh = AffineMesh(base, A, np.full(dim, 0.3))
    u = gi.linearization_point(mesh.n_nodes, dim, 1.5)
    om = orc.OracleMesh(mesh, np.zeros(mesh.n_nodes, np.uint8))
    o = orc.Oracle(om, theta=1.0, w0=1.0 / TAU, dt=TAU, order=1, consider_time_derivative=False,
                   increment_form=False, cell_wise_stabilization=True, **PRM)
    o._om = om
    o.set_linearization_point(u)
    return mesh, u, o


@pytest.mark.parametrize("dim,k,n_ref,A", CASES)
def test_kat4_matrix_based_equals_scaled_matrix_free(dim, k, n_ref, A):
    mesh, u, o = _setup(dim, k, n_ref, A)
    scale = np.tile(np.r_[np.full(dim, TAU), 1.0], (k + 1) ** dim)
    for c in range(mesh.n_cells):
        mb = matrix_based_cell(mesh, c, u, u)
        mf = o.cell_matrix(c)
        assert rel_err(mb, scale[:, None] * mf) < 1e-12, c


@pytest.mark.gpu
@pytest.mark.parametrize("dim,k,n_ref,A", CASES[:2])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_kat4_gpu_element_matrices(dim, k, n_ref, A, prec):
    import glsamd
    mesh, u, _ = _setup(dim, k, n_ref, A)
    op = glsamd.NavierStokesOperator(mesh, np.zeros(mesh.n_nodes, np.uint8), prec,
                                     brick=(0, 0, 0))
    op.set_parameters(theta=1.0, w0=1.0 / TAU, dt=TAU, order=1, consider_time_derivative=False,
                      increment_form=False, cell_wise_stabilization=True, **PRM)
    op.set_linearization_point(u)
    E = op.element_matrices()
    scale = np.tile(np.r_[np.full(dim, TAU), 1.0], (k + 1) ** dim)
    tol = 1e-12 if prec == "f64" else 2e-5
    for c in range(mesh.n_cells):
        assert rel_err(scale[:, None] * E[c], matrix_based_cell(mesh, c, u, u)) < tol, c
