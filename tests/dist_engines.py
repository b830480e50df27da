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
