"""TEST INFRASTRUCTURE: a CPU local-operator engine for glsdist (the oracle on
the rank-local mesh), so the partition / exchange logic runs with gloo on a
machine without a GPU.  Injected by the tests as glsdist's `engine`; never
imported by the product package, bench.py's timed path or smoke()."""
import numpy as np


class OracleEngine:
    """Local operator = the CPU oracle (oracle/liboracle.so) on the rank-local
    mesh, GpuEngine's interface (glsdist.GpuEngine)."""

    def __init__(self, lmesh, cmask, n_owned, precision="f64"):
        import torch
        import oracle as orc
        self.om = orc.OracleMesh(lmesh, cmask)
        self.orc = orc
        self.nc = lmesh.dim + 1
        self.n_owned_dofs = n_owned * self.nc
        cm = np.asarray(cmask[:n_owned], dtype=np.uint8)
        bits = (cm[:, None] >> np.arange(self.nc)[None, :]) & 1
        self.con = torch.from_numpy(np.flatnonzero(bits.ravel()))
        self.dtype = torch.float64
        self.device = "cpu"
        self.o = None

    def set_parameters(self, **params):
        self.o = self.orc.Oracle(self.om, **params)

    def set_linearization_point(self, v):
        self.o.set_linearization_point(v.numpy())

    def set_previous_solution(self, hist, w):
        self.o.set_previous_solution([h.numpy() for h in hist], w)

    def local_vmult(self, dst, src):
        import torch
        dst.copy_(torch.from_numpy(self.o.vmult(src.numpy())))

    def identity_rows(self, dst, src):
        dst[self.con] = src[self.con]

    def diagonal_raw(self, d):
        import torch
        d.copy_(torch.from_numpy(self.o.diagonal(self.n_owned_dofs // self.nc)))

    def invert_diagonal(self, d):
        import torch
        v = d.numpy()
        n = self.n_owned_dofs
        v[self.con.numpy()] = 1.0
        v[:] = np.where(np.abs(v) > 1e-10, 1.0 / np.where(v == 0, 1.0, v), 1.0)
        d.copy_(torch.from_numpy(v))


class OracleTransfers:
    """The owner-only lattice transfers of csrc/mg.hip (k_prolongate,
    k_restrict, k_interpolate) restated in numpy on rank-local level meshes
    and flagged child lattices (bit 31: not the owner cell), for the CPU
    tests of glsdist.DistributedMultigrid."""

    def __init__(self, dmg, meshes):
        self.dmg = dmg
        k, dim = meshes[0].degree, meshes[0].dim
        n, L = k + 1, 2 * k + 1
        nodes = [0.0, 0.5, 1.0] if k == 2 else [0.0, 1.0]
        P = np.zeros((L, n))
        for I in range(L):
            c = min(I // k, 1)
            xx = 0.5 * (c + nodes[I - c * k])
            for j in range(n):
                v = 1.0
                for mm in range(n):
                    if mm != j:
                        v *= (xx - nodes[mm]) / (nodes[j] - nodes[mm])
                P[I, j] = v
        self.P3 = P
        for _ in range(dim - 1):
            self.P3 = np.kron(P, self.P3)  # lexicographic, x fastest
        self.nc = dim + 1
        self.k, self.dim, self.L = k, dim, L

    def _level(self, l):
        D = self.dmg.levels[l]
        return D.r.lmesh.cell_nodes.astype(np.int64), D.r.eng.om.cmask

    def prolongate_add(self, l, dst_f, src_c):
        cn, ccm = self._level(l - 1)
        _, fcm = self._level(l)
        ch = self.dmg.child[l]
        own = (ch & 0x80000000) == 0
        fn = (ch & 0x7FFFFFFF).astype(np.int64)
        nc = self.nc
        src = src_c.numpy()
        out = dst_f.numpy()
        for comp in range(nc):
            u = src[cn * nc + comp] * (((ccm[cn] >> comp) & 1) == 0)
            v = u @ self.P3.T
            w = (((fcm[fn] >> comp) & 1) == 0) & own
            np.add.at(out, fn[w] * nc + comp, v[w])

    def restrict_add(self, l, dst_c, src_f):
        cn, ccm = self._level(l - 1)
        _, fcm = self._level(l)
        ch = self.dmg.child[l]
        own = (ch & 0x80000000) == 0
        fn = (ch & 0x7FFFFFFF).astype(np.int64)
        nc = self.nc
        src = src_f.numpy()
        out = dst_c.numpy()
        for comp in range(nc):
            w = (((fcm[fn] >> comp) & 1) == 0) & own
            v = np.where(w, src[fn * nc + comp], 0.0)
            u = v @ self.P3
            keep = ((ccm[cn] >> comp) & 1) == 0
            np.add.at(out, cn[keep] * nc + comp, u[keep])

    def interpolate(self, l, dst_c, src_f):
        cn, _ = self._level(l - 1)
        ch = self.dmg.child[l]
        fn = (ch & 0x7FFFFFFF).astype(np.int64)
        n, L, nc = self.k + 1, self.L, self.nc
        idx = []
        for i in range(n ** self.dim):
            ia = [i % n, (i // n) % n, i // (n * n)]
            idx.append(2 * ia[0] + L * (2 * ia[1] + (L * 2 * ia[2] if self.dim == 3 else 0)))
        src = src_f.numpy()
        out = dst_c.numpy()
        f = fn[:, idx]
        for comp in range(nc):
            out[cn * nc + comp] = src[f * nc + comp]



class OracleCoarseDirect:
    """Test twin of glsdist.RedundantCoarseLU: the whole coarse level on the
    oracle, its matrix assembled from unit vectors, dense solve (numpy)."""

    def __init__(self, mesh, cmask, precision):
        import oracle as orc
        self.om = orc.OracleMesh(mesh, cmask)
        self.A = None

    def setup(self, params, u, hist, weights):
        import oracle as orc
        o = orc.Oracle(self.om, **params)
        o.set_linearization_point(u.double().numpy())
        if hist is not None and params.get("order", 0) > 0:
            o.set_previous_solution([h.double().numpy() for h in hist], weights)
        n = self.om.n_dofs
        A = np.empty((n, n))
        e = np.zeros(n)
        for j in range(n):
            e[j] = 1.0
            A[:, j] = o.vmult(e)
            e[j] = 0.0
        self.A = A

    def solve(self, b):
        import torch
        return torch.from_numpy(np.linalg.solve(self.A, b.double().numpy())).to(b.dtype)
