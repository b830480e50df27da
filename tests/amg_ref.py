"""CPU restatement of the smoothed-aggregation AMG of csrc/amg.hip (test
infrastructure: the checker of gls_amg_*, not a product path).

The library's AMG substitutes TrilinosWrappers::PreconditionAMG (Trilinos
ML, multigrid.cc:372-433), which is not available here, so parity with ML
itself is unpinned; this file pins the GPU implementation to its own
published algorithm (csrc/amg.hip header): strength of connection on the
block node graph, three-pass standard aggregation, constant-mode tentative
prolongator, Jacobi-smoothed prolongator (omega 4/3 / lambda, 15 power
iterations from a fixed start vector), Galerkin R A P, dense coarsest solve,
Chebyshev smoothing of D^-1 A over [1.1 lambda / alpha, 1.1 lambda] (alpha 10:
the "smoother: Chebyshev alpha" deal.II passes to ML)."""
import numpy as np
import scipy.sparse as sp


def power_lambda(A, dinv):
    n = A.shape[0]
    i = np.arange(n, dtype=np.int64)
    x = 1.0 + ((i * 7919) % 97) / 97.0
    x /= np.linalg.norm(x)
    lam = 0.0
    for _ in range(15):
        y = dinv * (A @ x)
        lam = np.linalg.norm(y)
        if lam == 0:
            break
        x = y / lam
    return lam


def aggregate(A, b, theta):
    """agg[node], n_agg (the library's three passes, node order)."""
    N = A.shape[0] // b
    A2 = A.copy().tocoo()
    B = sp.csr_matrix((A2.data ** 2, (A2.row // b, A2.col // b)), shape=(N, N))
    B.sum_duplicates()
    B.sort_indices()
    B.data = np.sqrt(B.data)
    self_ = B.diagonal()
    S = []
    for I in range(N):
        cols = B.indices[B.indptr[I]:B.indptr[I + 1]]
        vals = B.data[B.indptr[I]:B.indptr[I + 1]]
        keep = (cols != I) & (vals > 0) & (vals >= theta * np.sqrt(self_[I] * self_[cols]))
        S.append(cols[keep])
    agg = np.full(N, -1, dtype=np.int64)
    # Dirichlet points (no off-diagonal entry): never aggregated (-2)
    for I in range(N):
        cols = B.indices[B.indptr[I]:B.indptr[I + 1]]
        if not np.any(cols != I):
            agg[I] = -2
    n_agg = 0
    for I in range(N):
        if agg[I] != -1:
            continue
        if np.any(agg[S[I]] >= 0):
            continue
        agg[I] = n_agg
        agg[S[I]] = n_agg
        n_agg += 1
    agg1 = agg.copy()
    for I in range(N):
        if agg1[I] < 0:
            for J in S[I]:
                if agg1[J] >= 0:
                    agg[I] = agg1[J]
                    break
    for I in range(N):
        if agg[I] != -1:
            continue
        agg[I] = n_agg
        for J in S[I]:
            if agg[J] < 0:
                agg[J] = n_agg
        n_agg += 1
    return agg, n_agg


class AMGRef:
    def __init__(self, A, block_size=1, threshold=1e-4, smoother_sweeps=2,
                 coarse_max_size=2000, elliptic=True, max_levels=10, chebyshev_alpha=10.0):
        self.sweeps = smoother_sweeps
        self.alpha = chebyshev_alpha if chebyshev_alpha > 0 else 10.0
        b = block_size
        A = sp.csr_matrix(A, dtype=np.float64)
        beta = np.ones(A.shape[0])
        self.levels = []
        lev = 0
        while True:
            d = A.diagonal()
            dinv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1.0), 1.0)
            lam = power_lambda(A, dinv)
            L = {"A": A, "dinv": dinv, "lam": lam}
            last = A.shape[0] <= coarse_max_size or lev + 1 >= max_levels
            if not last:
                agg, n_agg = aggregate(A, b, threshold)
                nc = n_agg * b
                if nc >= A.shape[0]:
                    self.levels.append(L)
                    break
                i = np.arange(A.shape[0])
                i = i[agg[i // b] >= 0]  # Dirichlet points: empty prolongator rows
                col = agg[i // b] * b + i % b
                nrm = np.sqrt(np.bincount(col, weights=beta[i] ** 2, minlength=nc))
                Pt = sp.csr_matrix((np.where(nrm[col] > 0, beta[i] / np.where(nrm[col] > 0, nrm[col], 1), 0),
                                    (i, col)), shape=(A.shape[0], nc))
                P = Pt
                if elliptic and lam > 0:
                    P = (Pt - sp.diags((4.0 / 3.0) / lam * dinv) @ (A @ Pt)).tocsr()
                R = P.T.tocsr()
                L["P"], L["R"] = P, R
                self.levels.append(L)
                A = (R @ (A @ P)).tocsr()
                beta = nrm
                lev += 1
                continue
            self.levels.append(L)
            break
        # coarsest above the library's dense limit (amg_dense_limit): smoothed
        n_last = self.levels[-1]["A"].shape[0]
        self.inv = (np.linalg.inv(self.levels[-1]["A"].toarray())
                    if n_last <= max(4 * coarse_max_size, 2048) else None)

    def _cheb(self, L, f, x):
        # s + 1 Chebyshev steps; the zero start (x None) skips the product A 0
        s = max(1, self.sweeps)
        b = 1.1 * L["lam"]
        a = b / self.alpha
        th, de = 0.5 * (b + a), 0.5 * (b - a)
        sg = th / de
        rho = 1.0 / sg
        A, dinv = L["A"], L["dinv"]
        if x is None:
            x = np.zeros_like(f)
            d = dinv * f / th
        else:
            d = dinv * (f - A @ x) / th
        for _ in range(s):
            rn = 1.0 / (2.0 * sg - rho)
            t = dinv * (f - A @ (x + d))
            x = x + d
            d = rn * rho * d + 2.0 * rn / de * t
            rho = rn
        return x + d

    def _vcycle(self, l, f):
        L = self.levels[l]
        if l + 1 == len(self.levels):
            return self.inv @ f if self.inv is not None else self._cheb(L, f, None)
        x = self._cheb(L, f, None)
        r = f - L["A"] @ x
        xc = self._vcycle(l + 1, L["R"] @ r)
        x = x + L["P"] @ xc
        return self._cheb(L, f, x)

    def vmult(self, src):
        return self._vcycle(0, np.asarray(src, dtype=np.float64))

    def info(self):
        return {"levels": len(self.levels),
                "sizes": [L["A"].shape[0] for L in self.levels],
                "lambda": [L["lam"] for L in self.levels]}
