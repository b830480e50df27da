"""TEST INFRASTRUCTURE: CPU multigrid on top of the oracle (oracle/liboracle.so)
— the restatement the GPU multigrid (csrc/mg.hip) is checked against.

Restates (deal.II semantics, not vendored; parity unpinned against the
reference binary):
  PreconditionRelaxation (relaxation = 0 -> power-iteration omega,
    deal.II's set_initial_guess / power_iteration / 1.2 safety factor),
    multigrid.cc:281-369: vmult (zero start) = x = w D^-1 b then n-1 steps,
    step = n times x += w D^-1 (b - A x)
  Multigrid::level_v_step V-cycle with MGSmootherPrecondition pre/post
    smoothing, MGTwoLevelTransfer restrict/prolongate (multigrid.cc:534-548)
  coarse solve: relaxation sweeps from zero (substitution for the
    Trilinos direct / AMG coarse solvers, multigrid.cc:448-489); with
    coarse_gmres_reltol, coarse_grid_iterate (multigrid.cc:491-530): deal.II
    SolverGMRES defaults (left preconditioning, restart after 28) under
    ReductionControl(10000, 1e-20, reltol), preconditioned by those sweeps
"""
import numpy as np

import oracle as orc


def power_start_vector(n_dofs, cmask, dim):
    """deal.II internal::PreconditionChebyshevImplementation::set_initial_guess
    (x_i = i % 11 on the global index, minus the mean) followed by
    AdditionalData::constraints.set_zero (multigrid.cc:302-303), normalised as
    power_iteration's first statement does.  deal.II >= 9.4, not vendored."""
    x = (np.arange(n_dofs) % 11).astype(np.float64)
    x -= x.mean()
    nc = dim + 1
    con = ((np.repeat(np.asarray(cmask, dtype=np.int64), nc)
            >> np.tile(np.arange(nc), len(cmask))) & 1).astype(bool)
    x[con] = 0.0
    return x / np.linalg.norm(x)


class OracleGMG:
    def __init__(self, meshes, cmasks, params, u_star, hist=None, weights=None,
                 n_smooth=5, n_eig=20, smoothing_range=20.0, coarse_iters=20,
                 coarse_gmres_reltol=None):
        self.meshes = meshes
        self.om = [orc.OracleMesh(m, c) for m, c in zip(meshes, cmasks)]
        self.omz = [orc.OracleMesh(m, np.zeros(m.n_nodes, np.uint8)) for m in meshes]
        self.child = [None] + [meshes[l - 1].child_lattice(meshes[l])
                               for l in range(1, len(meshes))]
        self.n_smooth, self.n_eig = n_smooth, n_eig
        self.range, self.coarse_iters = smoothing_range, coarse_iters
        self.coarse_gmres_reltol = coarse_gmres_reltol
        self.coarse_gmres_iterations = 0
        L = len(meshes)
        u = [None] * L
        h = [None] * L
        u[-1] = np.asarray(u_star, dtype=np.float64)
        h[-1] = None if hist is None else [np.asarray(x, dtype=np.float64) for x in hist]
        for l in range(L - 1, 0, -1):
            u[l - 1] = self.interpolate(l, u[l])
            if h[l] is not None:
                h[l - 1] = [self.interpolate(l, x) for x in h[l]]
        self.ops = []
        for l in range(L):
            o = orc.Oracle(self.om[l], **params)
            o.set_linearization_point(u[l])
            if h[l] is not None and params.get("order", 0) > 0:
                o.set_previous_solution(h[l], weights)
            self.ops.append(o)
        self.invdiag = [o.inverse_diagonal() for o in self.ops]
        self.omega = [1.0] * L
        self.lam = [0.0] * L

    def interpolate(self, l, fine):
        out = np.zeros(self.meshes[l - 1].n_dofs)
        orc.interpolate(self.omz[l - 1], self.omz[l], self.child[l], out, fine)
        return out

    def prolongate_add(self, l, dst_f, src_c):
        orc.prolongate_add(self.om[l - 1], self.om[l], self.child[l], dst_f, src_c)

    def restrict_add(self, l, dst_c, src_f):
        orc.restrict_add(self.om[l - 1], self.om[l], self.child[l], dst_c, src_f)

    def estimate(self, l):
        """max_eigenvalue_estimate of PreconditionRelaxation::estimate_eigenvalues
        with EigenvalueAlgorithm::power_iteration: |x . D^-1 A x| of the
        normalised iterate after n_eig steps, times the 1.2 safety factor."""
        m = self.meshes[l]
        x = power_start_vector(m.n_dofs, self.om[l].cmask, m.dim)
        lam = 0.0
        for _ in range(self.n_eig):
            y = self.invdiag[l] * self.ops[l].vmult(x)
            lam = float(x @ y)
            ny = np.linalg.norm(y)
            x = y / ny if ny > 0 else 0.0 * y
        return 1.2 * abs(lam)

    def set_omega(self, omegas):
        self.omega = list(omegas)

    def setup_omega(self):
        for l in range(len(self.ops)):
            ev_max = self.estimate(l)
            self.lam[l] = ev_max
            alpha = ev_max / self.range if self.range > 1 else 0.9 * ev_max
            self.omega[l] = 2.0 / (alpha + ev_max) if ev_max > 0 else 1.0

    def smooth(self, l, x, b, zero_start, iters):
        w, d, A = self.omega[l], self.invdiag[l], self.ops[l]
        it = 0
        if zero_start and iters > 0:
            x = w * d * b
            it = 1
        for _ in range(it, iters):
            x = x + w * d * (b - A.vmult(x))
        return x

    def coarse_matrix(self):
        """The assembled coarse operator (dense, FP64): the oracle's element
        matrices (orc_cell_matrix: unit-vector cell applies,
        MatrixFreeTools::compute_matrix, operator_ns.cc:1407-1430) summed
        over the cells on the free dofs; constrained rows and columns are the
        unit vector (identity rows of vmult, homogeneous constraints read as
        0).  Equal to the matrix of the oracle's vmult (test_mg_ref.py)."""
        if not hasattr(self, "_A0"):
            m, o = self.om[0], self.ops[0]
            nc = m.dim + 1
            n = m.n_dofs
            con = ((np.repeat(m.cmask.astype(np.int64), nc) >>
                    np.tile(np.arange(nc), m.n_nodes)) & 1).astype(bool)
            A = np.zeros((n, n))
            for c in range(m.n_cells):
                dofs = (m.cell_nodes[c].astype(np.int64)[:, None] * nc +
                        np.arange(nc)[None, :]).reshape(-1)
                A[np.ix_(dofs, dofs)] += o.cell_matrix(c)
            A[con, :] = 0.0
            A[:, con] = 0.0
            A[con, con] = 1.0
            self._A0 = A
            self._con0 = con
        return self._A0

    def coarse_direct(self, b):
        """Direct coarse solve (the decks' "direct", multigrid.cc:448-455):
        x_c = b_c on the constrained dofs, LU of the free block for the rest
        (the factorisation cached)."""
        import scipy.linalg as sla
        if not hasattr(self, "_lu0"):
            A = self.coarse_matrix()
            free = ~self._con0
            self._lu0 = sla.lu_factor(A[np.ix_(free, free)], check_finite=False)
            self._free0 = free
        x = np.asarray(b, dtype=np.float64).copy()
        x[self._free0] = sla.lu_solve(self._lu0, x[self._free0], check_finite=False)
        return x

    def coarse_precondition(self, b):
        if self.coarse_iters < 0:
            return self.coarse_direct(b)
        if self.coarse_iters == 0:
            return b.copy()
        return self.smooth(0, None, b, True, self.coarse_iters)

    def coarse_gmres(self, b, m=28, maxiter=10000):
        A, P = self.ops[0].vmult, self.coarse_precondition
        x = np.zeros_like(b)
        r = P(b)
        res = np.linalg.norm(r)
        tol = max(self.coarse_gmres_reltol * res, 1e-20)
        it = 0
        while res > tol and it < maxiter:
            V = [r / res]
            H = np.zeros((m + 1, m))
            g = np.zeros(m + 1)
            g[0] = res
            cs, sn = np.zeros(m), np.zeros(m)
            jd = 0
            for j in range(m):
                w = P(A(V[j]))
                h = np.zeros(j + 1)
                for _ in range(2):  # CGS2
                    hp = np.array([v @ w for v in V])
                    w = w - sum(c * v for c, v in zip(hp, V))
                    h += hp
                hn = np.linalg.norm(w)
                H[:j + 1, j] = h
                H[j + 1, j] = hn
                V.append(w / hn if hn > 0 else w)
                for i in range(j):
                    t = cs[i] * H[i, j] + sn[i] * H[i + 1, j]
                    H[i + 1, j] = -sn[i] * H[i, j] + cs[i] * H[i + 1, j]
                    H[i, j] = t
                rr = np.hypot(H[j, j], H[j + 1, j])
                cs[j], sn[j] = (H[j, j] / rr, H[j + 1, j] / rr) if rr > 0 else (1.0, 0.0)
                H[j, j], H[j + 1, j] = rr, 0.0
                g[j + 1] = -sn[j] * g[j]
                g[j] = cs[j] * g[j]
                it += 1
                jd += 1
                res = abs(g[j + 1])
                if res <= tol or hn == 0:
                    break
            y = np.zeros(jd)
            for i in range(jd - 1, -1, -1):
                y[i] = (g[i] - H[i, i + 1:jd] @ y[i + 1:jd]) / H[i, i]
            x = x + sum(c * v for c, v in zip(y, V[:jd]))
            if res <= tol:
                break
            r = P(b - A(x))
            res = np.linalg.norm(r)
        self.coarse_gmres_iterations = it
        return x

    def v_step(self, l, b):
        if l == 0 and self.coarse_gmres_reltol is not None:
            return self.coarse_gmres(b)
        if l == 0:
            return self.coarse_precondition(b)
        x = self.smooth(l, None, b, True, self.n_smooth)
        t = b - self.ops[l].vmult(x)
        bc = np.zeros(self.meshes[l - 1].n_dofs)
        self.restrict_add(l, bc, t)
        xc = self.v_step(l - 1, bc)
        x = x.copy()
        self.prolongate_add(l, x, xc)
        return self.smooth(l, x, b, False, self.n_smooth)

    def vcycle(self, b):
        return self.v_step(len(self.ops) - 1, np.asarray(b, dtype=np.float64))
