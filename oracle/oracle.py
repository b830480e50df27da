"""TEST INFRASTRUCTURE ONLY — ctypes binding of oracle/liboracle.so.

The CPU restatement of the reference hot path (see gls_oracle.h for the
reference lines it follows and its parity status: pinned by KAT-1..6,
"parity unpinned" against the reference binary, which cannot be built here).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class _Mesh(C.Structure):
    _fields_ = [("dim", C.c_int), ("degree", C.c_int), ("n_cells", C.c_int64),
                ("n_nodes", C.c_int64), ("cell_nodes", C.c_void_p), ("coords", C.c_void_p),
                ("cmask", C.c_void_p), ("cell_measure", C.c_void_p), ("cell_hmin", C.c_void_p),
                ("mapping_degree", C.c_int), ("mapping_points", C.c_void_p)]


class _Params(C.Structure):
    _fields_ = [("nu", C.c_double), ("c1", C.c_double), ("c2", C.c_double),
                ("theta", C.c_double), ("w0", C.c_double), ("dt", C.c_double),
                ("order", C.c_int), ("consider_time_derivative", C.c_int),
                ("increment_form", C.c_int), ("cell_wise_stabilization", C.c_int)]


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        vp = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(_Mesh), C.POINTER(_Params)]
        L.orc_create.restype = vp
        L.orc_destroy.argtypes = [vp]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_set_linearization_point.argtypes = [vp, vp]
        L.orc_set_previous_solution.argtypes = [vp, vp, C.c_int, vp]
        L.orc_vmult.argtypes = [vp, vp, vp]
        L.orc_evaluate_residual.argtypes = [vp, vp, vp]
        L.orc_compute_inverse_diagonal.argtypes = [vp, vp]
        L.orc_compute_diagonal.argtypes = [vp, C.c_int64, vp]
        L.orc_get_max_u.argtypes = [vp, vp]
        L.orc_get_max_u.restype = C.c_double
        L.orc_cell_matrix.argtypes = [vp, C.c_int64, vp]
        L.orc_set_outflow_faces.argtypes = [vp, C.c_int64, vp, vp, vp]
        L.orc_set_outflow_faces.restype = C.c_int
        L.orc_outflow_face_points.argtypes = [vp, vp]
        L.orc_set_outflow_target.argtypes = [vp, vp]
        L.orc_get_tables.argtypes = [vp, vp, vp]
        L.orc_get_tables.restype = C.c_int
        L.orc_get_geometry.argtypes = [vp, vp]
        L.orc_bdf_weights.argtypes = [C.c_int, vp, vp]
        L.orc_bdf_weights.restype = C.c_int
        for f in ("orc_prolongate_add", "orc_restrict_add", "orc_interpolate"):
            getattr(L, f).argtypes = [vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def set_threads(n):
    lib().orc_set_threads(int(n))


def _p(a):
    return a.ctypes.data


class OracleMesh:
    """Holds the numpy arrays alive for an orc_mesh struct."""

    def __init__(self, mesh, cmask):
        self.dim = mesh.dim
        self.degree = mesh.degree
        self.n_nodes = mesh.n_nodes
        self.n_cells = mesh.n_cells
        self.cell_nodes = np.ascontiguousarray(mesh.cell_nodes, dtype=np.uint32)
        self.coords = np.ascontiguousarray(mesh.coords, dtype=np.float64)
        self.cmask = np.ascontiguousarray(cmask, dtype=np.uint8)
        meas, hmin = mesh.cell_measure()
        self.measure = np.ascontiguousarray(meas)
        self.hmin = np.ascontiguousarray(hmin)
        # MappingQ_m of another degree (the FE_Q_iso_Q1 level's parent mapping)
        mp = getattr(mesh, "mapping_points", None)
        self.mapping = mp() if callable(mp) else None
        mdeg, mptr = 0, None
        if self.mapping is not None:
            mdeg, pts = self.mapping
            self.mapping_pts = np.ascontiguousarray(pts, dtype=np.float64)
            mptr = _p(self.mapping_pts)
        self.s = _Mesh(self.dim, self.degree, self.n_cells, self.n_nodes, _p(self.cell_nodes),
                       _p(self.coords), _p(self.cmask), _p(self.measure), _p(self.hmin),
                       mdeg, mptr)

    @property
    def n_dofs(self):
        return self.n_nodes * (self.dim + 1)


class Oracle:
    """CPU NavierStokesOperator restatement on one mesh (double precision)."""

    def __init__(self, omesh: OracleMesh, nu, c1=1.0, c2=1.0, theta=1.0, w0=0.0, dt=1.0,
                 order=0, consider_time_derivative=False, increment_form=True,
                 cell_wise_stabilization=False):
        self.m = omesh
        self.prm = _Params(nu, c1, c2, theta, w0, dt, order, int(consider_time_derivative),
                           int(increment_form), int(cell_wise_stabilization))
        self.h = lib().orc_create(C.byref(omesh.s), C.byref(self.prm))
        if not self.h:
            raise RuntimeError("orc_create failed")
        self.nq = (omesh.degree + 1) ** omesh.dim

    def __del__(self):
        try:
            lib().orc_destroy(self.h)
        except Exception:
            pass

    def set_outflow_faces(self, cells, face_no, kind):
        """Outflow boundary faces (orc_set_outflow_faces); kind "cut" /
        "nitsche" or a per-face array of 1 / 2."""
        cells = np.ascontiguousarray(cells, dtype=np.int64)
        face_no = np.ascontiguousarray(face_no, dtype=np.int32)
        if isinstance(kind, str):
            kind = np.full(len(cells), {"cut": 1, "nitsche": 2}[kind], dtype=np.int32)
        kind = np.ascontiguousarray(kind, dtype=np.int32)
        self._faces = (cells, face_no, kind)
        if lib().orc_set_outflow_faces(self.h, len(cells), _p(cells), _p(face_no), _p(kind)):
            raise ValueError("orc_set_outflow_faces: bad faces")
        self.n_faces = len(cells)
        self.nqf = (self.m.degree + 1) ** (self.m.dim - 1)

    def outflow_face_points(self):
        x = np.empty((self.n_faces, self.nqf, self.m.dim))
        lib().orc_outflow_face_points(self.h, _p(x))
        return x

    def set_outflow_target(self, target):
        t = np.ascontiguousarray(target, dtype=np.float64)
        assert t.size == self.n_faces * self.nqf * self.m.dim
        lib().orc_set_outflow_target(self.h, _p(t))

    def set_linearization_point(self, vec):
        vec = np.ascontiguousarray(vec, dtype=np.float64)
        lib().orc_set_linearization_point(self.h, _p(vec))

    def set_previous_solution(self, history, weights):
        hist = [np.ascontiguousarray(h, dtype=np.float64) for h in history]
        ptrs = (C.c_void_p * len(hist))(*[_p(h) for h in hist])
        w = np.ascontiguousarray(weights, dtype=np.float64)
        lib().orc_set_previous_solution(self.h, C.cast(ptrs, C.c_void_p), len(hist), _p(w))

    def vmult(self, src):
        src = np.ascontiguousarray(src, dtype=np.float64)
        dst = np.empty_like(src)
        lib().orc_vmult(self.h, _p(dst), _p(src))
        return dst

    def evaluate_residual(self, src):
        src = np.ascontiguousarray(src, dtype=np.float64)
        dst = np.empty_like(src)
        lib().orc_evaluate_residual(self.h, _p(dst), _p(src))
        return dst

    def get_max_u(self, vec):
        vec = np.ascontiguousarray(vec, dtype=np.float64)
        return float(lib().orc_get_max_u(self.h, _p(vec)))

    def diagonal(self, n_owned_nodes=None):
        """Assembled diagonal before inversion (partitioned operators)."""
        d = np.empty(self.m.n_dofs)
        lib().orc_compute_diagonal(self.h, self.m.n_nodes if n_owned_nodes is None
                                   else int(n_owned_nodes), _p(d))
        return d

    def inverse_diagonal(self):
        d = np.empty(self.m.n_dofs)
        lib().orc_compute_inverse_diagonal(self.h, _p(d))
        return d

    def cell_matrix(self, cell):
        nd = self.nq * (self.m.dim + 1)
        A = np.empty((nd, nd))
        lib().orc_cell_matrix(self.h, int(cell), _p(A))
        return A

    def tables(self):
        dim = self.m.dim
        nf = 2 + 3 * dim + dim * dim
        t = np.empty((self.m.n_cells, self.nq, nf))
        cw = np.empty((self.m.n_cells, 2))
        lib().orc_get_tables(self.h, _p(t), _p(cw))
        return t, cw

    def geometry(self):
        dim = self.m.dim
        g = np.empty((self.m.n_cells, self.nq, 1 + dim * dim))
        lib().orc_get_geometry(self.h, _p(g))
        return g


def bdf_weights(order, dts):
    dt = np.zeros(max(order, 1))
    dt[:len(dts)] = dts[:order]
    w = np.zeros(order + 1)
    lib().orc_bdf_weights(order, _p(dt), _p(w))
    return w


def prolongate_add(cm: OracleMesh, fm: OracleMesh, child, dst_f, src_c):
    child = np.ascontiguousarray(child, dtype=np.uint32)
    src_c = np.ascontiguousarray(src_c, dtype=np.float64)
    lib().orc_prolongate_add(C.byref(cm.s), C.byref(fm.s), _p(child), _p(dst_f), _p(src_c))


def restrict_add(cm: OracleMesh, fm: OracleMesh, child, dst_c, src_f):
    child = np.ascontiguousarray(child, dtype=np.uint32)
    src_f = np.ascontiguousarray(src_f, dtype=np.float64)
    lib().orc_restrict_add(C.byref(cm.s), C.byref(fm.s), _p(child), _p(dst_c), _p(src_f))


def interpolate(cm: OracleMesh, fm: OracleMesh, child, dst_c, src_f):
    child = np.ascontiguousarray(child, dtype=np.uint32)
    src_f = np.ascontiguousarray(src_f, dtype=np.float64)
    lib().orc_interpolate(C.byref(cm.s), C.byref(fm.s), _p(child), _p(dst_c), _p(src_f))


# ------------------------------------------------------------ batched CPU port
def cpu_isa():
    """'avx512' or 'avx2' from the host CPU flags (the batched build to load)."""
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        flags = ""
    return "avx512" if " avx512f" in flags and " avx512dq" in flags else "avx2"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class BatchedCPU:
    """The cell-batched SIMD CPU restatement (oracle/gls_cpu_batched.c) of the
    headline Newton vmult (3D Q2, q-wise stabilisation), built from an Oracle's
    tables and geometry on the same mesh: bench.py's cpu_baseline."""

    def __init__(self, o: Oracle, threads):
        m = o.m
        if m.dim != 3 or m.degree != 2 or not o.prm.increment_form or o.prm.cell_wise_stabilization:
            raise ValueError("BatchedCPU: 3D Q2 Newton operator with q-wise delta only")
        self.isa = cpu_isa()
        L = C.CDLL(os.path.join(_HERE, f"libcpu_batched_{self.isa}.so"))
        vp = C.c_void_p
        L.cpu_create.argtypes = [C.c_int64, C.c_int64, vp, vp, vp, vp, C.c_double, C.c_double,
                                 C.c_int, C.c_int]
        L.cpu_create.restype = vp
        L.cpu_vmult.argtypes = [vp, vp, vp]
        L.cpu_destroy.argtypes = [vp]
        L.cpu_n_colors.argtypes = [vp]
        self.L = L
        t, _ = o.tables()
        g = o.geometry()
        td = int(o.prm.consider_time_derivative and o.prm.order > 0)
        self.threads = int(threads)
        self.h = L.cpu_create(m.n_cells, m.n_nodes, _p(m.cell_nodes), _p(m.cmask), _p(g), _p(t),
                              o.prm.nu, o.prm.w0, td, self.threads)
        self.n_colors = L.cpu_n_colors(self.h)
        self.n_dofs = m.n_dofs

    def __del__(self):
        try:
            self.L.cpu_destroy(self.h)
        except Exception:
            pass

    def vmult(self, src, dst=None):
        src = np.ascontiguousarray(src, dtype=np.float64)
        if dst is None:
            dst = np.empty_like(src)
        self.L.cpu_vmult(self.h, _p(dst), _p(src))
        return dst
