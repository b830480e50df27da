"""ctypes binding of libglsamd.so (include/gls_op.h) — Python mirror of the
reference's OperatorBase<Number> interface (include/operator_base.h:13-73)
for the matrix-free GLS Navier–Stokes operator on MI355X.

Vectors are torch tensors on the GPU (torch is plumbing: device memory and
streams); every compute call goes through the HIP kernels of libglsamd.so.
There is no CPU fallback: a missing library or GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.normpath(os.path.join(_HERE, "..", "lib"))
_lib = None

GLS_F64, GLS_F32 = 0, 1
GLS_INCREMENT_FORM, GLS_CONSIDER_TIME_DERIVATIVE, GLS_CELL_WISE_STAB = 1, 2, 4
GLS_DETERMINISTIC = 8

# exported symbols of include/gls_op.h (checked by tests/test_abi.py)
EXPORTS = [
    "gls_op_create", "gls_op_destroy", "gls_op_set_parameters", "gls_op_m",
    "gls_op_precision", "gls_op_set_linearization_point", "gls_op_set_previous_solution",
    "gls_op_vmult", "gls_op_vmult_interface_down", "gls_op_vmult_interface_up",
    "gls_op_vmult_cells", "gls_op_vmult_init", "gls_op_apply_identity_rows",
    "gls_op_evaluate_residual", "gls_op_evaluate_residual_plain", "gls_op_evaluate_rhs",
    "gls_op_set_constraint_values", "gls_gmres_solve",
    "gls_op_compute_inverse_diagonal", "gls_op_upload_tables", "gls_op_download_tables",
    "gls_op_geometry_counts", "gls_op_vmult_bytes", "gls_mg_create", "gls_mg_destroy",
    "gls_mg_setup", "gls_mg_get_relaxation", "gls_mg_vcycle", "gls_mg_prolongate_add",
    "gls_mg_restrict_add", "gls_mg_interpolate", "gls_mg_smooth", "gls_last_error",
    "gls_dist_unique_id", "gls_dist_create", "gls_dist_destroy", "gls_dist_vmult",
    "gls_dist_vmult_group", "gls_dist_interior_bricks", "gls_op_set_vector_layout",
    "gls_op_get_max_u", "gls_mg_set_vector_layout", "gls_dist_update_ghost_values",
    "gls_dist_get_max_u", "gls_op_compute_diagonal", "gls_op_invert_diagonal", "gls_mg_relax",
    "gls_dist_compress_add", "gls_op_brick_shape", "gls_op_sweep_stats", "gls_op_cell_permutation",
    "gls_op_set_sweep_spin_bound",
    "gls_timer_enable", "gls_timer_reset", "gls_timer_n_sections", "gls_timer_section",
    "gls_timer_report", "gls_timer_begin", "gls_timer_end",
    "gls_discover_bricks", "gls_mg_coarse_statistics", "gls_mg_coarse_setup_times",
    "gls_amg_create", "gls_amg_destroy", "gls_amg_vmult", "gls_amg_info", "gls_mg_coarse_amg",
    "gls_amg_level_matrix",
    "gls_dist_mg_create", "gls_dist_mg_destroy", "gls_dist_mg_set_linearization_point",
    "gls_dist_mg_setup", "gls_dist_mg_get_relaxation", "gls_dist_mg_vcycle",
    "gls_dist_gmres_solve", "gls_op_element_matrices",
    "gls_op_system_matrix", "gls_op_n_outflow_faces", "gls_op_outflow_face_points",
    "gls_op_set_outflow_target",
]

GLS_MEM_DEVICE, GLS_MEM_HOST = 0, 1


class OpDesc(C.Structure):
    _fields_ = [("dim", C.c_int), ("degree", C.c_int), ("precision", C.c_int),
                ("n_cells", C.c_int64), ("n_nodes", C.c_int64), ("n_owned_nodes", C.c_int64),
                ("cell_nodes", C.c_void_p), ("node_coords", C.c_void_p),
                ("node_cmask", C.c_void_p), ("cell_measure", C.c_void_p),
                ("cell_hmin", C.c_void_p), ("brick", C.c_int * 3),
                ("n_outflow_faces", C.c_int64), ("outflow_cells", C.c_void_p),
                ("outflow_face_no", C.c_void_p), ("outflow_kind", C.c_void_p),
                ("mapping_degree", C.c_int), ("mapping_points", C.c_void_p)]

OUTFLOW_KIND = {"cut": 1, "nitsche": 2}


class OpParams(C.Structure):
    _fields_ = [("nu", C.c_double), ("c1", C.c_double), ("c2", C.c_double),
                ("theta", C.c_double), ("w0", C.c_double), ("dt", C.c_double),
                ("order", C.c_int), ("flags", C.c_int)]


class AMGParams(C.Structure):
    _fields_ = [("block_size", C.c_int), ("threshold", C.c_double),
                ("smoother_sweeps", C.c_int), ("coarse_max_size", C.c_int),
                ("elliptic", C.c_int), ("max_levels", C.c_int),
                ("chebyshev_alpha", C.c_double)]


def amg_params(block_size=1, threshold=1e-4, smoother_sweeps=2, coarse_max_size=2000,
               elliptic=True, max_levels=10, chebyshev_alpha=10.0):
    """glsAMGParams; the defaults are TrilinosWrappers::PreconditionAMG::
    AdditionalData()'s (one constant mode, threshold 1e-4, 2 smoother sweeps,
    elliptic) with the ML parameters deal.II sets ("coarse: max size" 2000,
    "smoother: Chebyshev alpha" 10)."""
    return AMGParams(int(block_size), float(threshold), int(smoother_sweeps),
                     int(coarse_max_size), int(bool(elliptic)), int(max_levels),
                     float(chebyshev_alpha))


class MGDesc(C.Structure):
    _fields_ = [("n_levels", C.c_int), ("smoothing_n_iterations", C.c_int),
                ("smoothing_eig_n_iterations", C.c_int), ("smoothing_range", C.c_double),
                ("coarse_n_iterations", C.c_int), ("outer_precision", C.c_int),
                ("compute_evs_n_levels", C.c_int), ("coarse_iterate", C.c_int),
                ("coarse_reltol", C.c_double), ("coarse_maxiter", C.c_int),
                ("coarse_amg", C.c_int), ("amg", AMGParams)]


class DistDesc(C.Structure):
    _fields_ = [("rank", C.c_int), ("world", C.c_int), ("nccl_id", C.c_void_p),
                ("group", C.c_void_p), ("n_peers", C.c_int), ("peers", C.c_void_p),
                ("send_count", C.c_void_p), ("send_nodes", C.c_void_p),
                ("recv_begin", C.c_void_p), ("recv_count", C.c_void_p)]


class GMRESDesc(C.Structure):
    _fields_ = [("max_n_tmp_vectors", C.c_int), ("max_iterations", C.c_int),
                ("absolute_tolerance", C.c_double), ("relative_tolerance", C.c_double)]


class GMRESResult(C.Structure):
    _fields_ = [("n_iterations", C.c_int), ("n_restarts", C.c_int), ("converged", C.c_int),
                ("initial_residual", C.c_double), ("final_residual", C.c_double),
                ("tolerance", C.c_double)]


def lib_path():
    return os.path.join(LIBDIR, "libglsamd.so")


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("GLS_AMD_LIB") or lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make amd` (or __graft_entry__.build())")
        L = C.CDLL(path)
        vp, i64 = C.c_void_p, C.c_int64
        L.gls_op_create.argtypes = [C.POINTER(OpDesc), C.POINTER(vp)]
        L.gls_op_destroy.argtypes = [vp]
        L.gls_op_set_parameters.argtypes = [vp, C.POINTER(OpParams)]
        L.gls_op_m.argtypes = [vp]
        L.gls_op_m.restype = i64
        L.gls_op_precision.argtypes = [vp]
        L.gls_op_set_linearization_point.argtypes = [vp, vp, vp]
        L.gls_op_set_previous_solution.argtypes = [vp, vp, C.c_int, vp, vp]
        L.gls_op_vmult.argtypes = [vp, vp, vp, vp]
        L.gls_op_vmult_interface_down.argtypes = [vp, vp, vp, vp]
        L.gls_op_vmult_interface_up.argtypes = [vp, vp, vp, vp]
        L.gls_op_vmult_cells.argtypes = [vp, vp, vp, i64, i64, vp]
        L.gls_op_vmult_init.argtypes = [vp, vp, vp, vp]
        L.gls_op_apply_identity_rows.argtypes = [vp, vp, vp, vp]
        L.gls_op_evaluate_residual.argtypes = [vp, vp, vp, vp]
        L.gls_op_evaluate_residual_plain.argtypes = [vp, vp, vp, vp]
        L.gls_op_evaluate_rhs.argtypes = [vp, vp, vp]
        L.gls_op_set_constraint_values.argtypes = [vp, vp, vp]
        L.gls_op_compute_inverse_diagonal.argtypes = [vp, vp, vp]
        L.gls_op_upload_tables.argtypes = [vp, vp, vp]
        L.gls_op_download_tables.argtypes = [vp, vp, vp]
        L.gls_op_geometry_counts.argtypes = [vp, C.POINTER(i64), C.POINTER(i64)]
        L.gls_op_vmult_bytes.argtypes = [vp]
        L.gls_op_vmult_bytes.restype = C.c_double
        L.gls_mg_create.argtypes = [C.POINTER(MGDesc), vp, vp, C.POINTER(vp)]
        L.gls_mg_destroy.argtypes = [vp]
        L.gls_mg_setup.argtypes = [vp, vp]
        L.gls_mg_get_relaxation.argtypes = [vp, C.c_int, C.POINTER(C.c_double),
                                            C.POINTER(C.c_double)]
        L.gls_mg_vcycle.argtypes = [vp, vp, vp, vp]
        for f in ("gls_mg_prolongate_add", "gls_mg_restrict_add", "gls_mg_interpolate"):
            getattr(L, f).argtypes = [vp, C.c_int, vp, vp, vp]
        L.gls_mg_smooth.argtypes = [vp, C.c_int, vp, vp, C.c_int, vp]
        L.gls_dist_unique_id.argtypes = [vp]
        L.gls_dist_create.argtypes = [vp, C.POINTER(DistDesc), C.POINTER(vp)]
        L.gls_dist_destroy.argtypes = [vp]
        L.gls_dist_vmult.argtypes = [vp, vp, vp, vp]
        L.gls_dist_vmult_group.argtypes = [vp, vp, vp, C.c_int, vp]
        L.gls_dist_interior_bricks.argtypes = [vp, C.POINTER(i64), C.POINTER(i64)]
        L.gls_gmres_solve.argtypes = [vp, vp, C.POINTER(GMRESDesc), vp, vp,
                                      C.POINTER(GMRESResult), vp]
        L.gls_op_set_vector_layout.argtypes = [vp, C.c_int, vp]
        L.gls_op_get_max_u.argtypes = [vp, vp, C.POINTER(C.c_double), vp]
        L.gls_mg_set_vector_layout.argtypes = [vp, C.c_int, vp]
        L.gls_dist_update_ghost_values.argtypes = [vp, vp, vp]
        L.gls_dist_get_max_u.argtypes = [vp, vp, C.POINTER(C.c_double), vp]
        L.gls_op_compute_diagonal.argtypes = [vp, vp, vp]
        L.gls_op_invert_diagonal.argtypes = [vp, vp, vp]
        L.gls_mg_relax.argtypes = [vp, C.c_int, vp, vp, vp, vp, C.c_double, C.c_int, vp]
        L.gls_dist_compress_add.argtypes = [vp, vp, vp]
        L.gls_op_brick_shape.argtypes = [vp, vp]
        L.gls_op_sweep_stats.argtypes = [vp, vp, vp]
        L.gls_op_set_sweep_spin_bound.argtypes = [vp, C.c_int64]
        L.gls_op_cell_permutation.argtypes = [vp, vp]
        L.gls_op_element_matrices.argtypes = [vp, vp]
        L.gls_op_system_matrix.argtypes = [vp, C.POINTER(i64), vp, vp, vp]
        L.gls_op_n_outflow_faces.argtypes = [vp, C.POINTER(i64), C.POINTER(C.c_int)]
        L.gls_op_outflow_face_points.argtypes = [vp, vp]
        L.gls_op_set_outflow_target.argtypes = [vp, vp, vp]
        L.gls_mg_coarse_statistics.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.gls_mg_coarse_setup_times.argtypes = [vp, vp, C.POINTER(C.c_int)]
        L.gls_amg_create.argtypes = [i64, vp, vp, vp, C.POINTER(AMGParams), C.POINTER(vp)]
        L.gls_amg_destroy.argtypes = [vp]
        L.gls_amg_destroy.restype = None
        L.gls_amg_vmult.argtypes = [vp, vp, vp, vp]
        L.gls_amg_info.argtypes = [vp, C.POINTER(C.c_int), vp, vp, vp]
        L.gls_amg_level_matrix.argtypes = [vp, C.c_int, C.c_int, C.POINTER(i64), C.POINTER(i64),
                                           vp, vp, vp]
        L.gls_mg_coarse_amg.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_double)]
        L.gls_dist_mg_create.argtypes = [vp, vp, vp]
        L.gls_dist_mg_destroy.argtypes = [vp]
        L.gls_dist_mg_destroy.restype = None
        L.gls_dist_mg_set_linearization_point.argtypes = [vp, C.c_int, vp, vp, C.c_int, vp, vp]
        L.gls_dist_mg_setup.argtypes = [vp, C.c_int, vp]
        L.gls_dist_mg_get_relaxation.argtypes = [vp, C.c_int, C.POINTER(C.c_double),
                                                 C.POINTER(C.c_double)]
        L.gls_dist_mg_vcycle.argtypes = [vp, C.c_int, vp, vp, vp]
        L.gls_dist_gmres_solve.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp]
        L.gls_discover_bricks.argtypes = [C.c_int, C.c_int, i64, vp, vp, vp]
        L.gls_last_error.restype = C.c_char_p
        L.gls_timer_enable.argtypes = [C.c_int, C.POINTER(C.c_int)]
        L.gls_timer_reset.argtypes = []
        L.gls_timer_n_sections.argtypes = []
        L.gls_timer_n_sections.restype = i64
        L.gls_timer_section.argtypes = [i64, C.c_char_p, i64, C.POINTER(i64),
                                        C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.gls_timer_begin.argtypes = [C.c_char_p, vp, C.POINTER(vp)]
        L.gls_timer_end.argtypes = [vp]
        L.gls_timer_report.argtypes = [C.c_char_p, i64]
        L.gls_timer_report.restype = i64
        _lib = L
    return _lib


class GlsError(RuntimeError):
    pass


# ---- timer sections (gls_timer_*: MyTimerOutput / MyScope, timer.h:194-413)
def timer_enable(on=True):
    """Tally the library's timer sections (host wall time and GPU time
    between events on each section's stream); returns the previous state.
    Sections are roctx ranges either way."""
    was = C.c_int(0)
    _check(lib().gls_timer_enable(1 if on else 0, C.byref(was)))
    return bool(was.value)


def timer_reset():
    _check(lib().gls_timer_reset())


def timer_sections():
    """{name: {"calls", "host_ms", "gpu_ms"}} (gpu_ms None without events);
    reading waits for the sections' pending events."""
    L = lib()
    out = {}
    name = C.create_string_buffer(256)
    for i in range(L.gls_timer_n_sections()):
        calls, hms, gms = C.c_int64(0), C.c_double(0), C.c_double(0)
        _check(L.gls_timer_section(i, name, 256, C.byref(calls), C.byref(hms), C.byref(gms)))
        out[name.value.decode()] = {"calls": calls.value, "host_ms": hms.value,
                                    "gpu_ms": gms.value if gms.value >= 0 else None}
    return out


class timer_scope:
    """MyScope (timer.h:342-413) around the caller's own code: a timer
    section (roctx range; tallied when timing is on) on torch's current
    stream, e.g. `with glsamd.timer_scope("newton::solve"): ...`."""

    def __init__(self, name, stream=None):
        self.name, self.stream = name.encode(), stream
        self.tok = C.c_void_p()

    def __enter__(self):
        s = self.stream if self.stream is not None else _stream_or_null()
        _check(lib().gls_timer_begin(self.name, s, C.byref(self.tok)))
        return self

    def __exit__(self, *exc):
        _check(lib().gls_timer_end(self.tok))
        return False


def _stream_or_null():
    try:
        import torch
        if torch.cuda.is_available():
            return _stream()
    except ImportError:
        pass
    return None


def timer_report():
    """The tally as TimerOutput-style text (print_wall_time_statistics)."""
    L = lib()
    n = L.gls_timer_report(None, 0)
    buf = C.create_string_buffer(int(n))
    L.gls_timer_report(buf, n)
    return buf.value.decode()


def _check(rc):
    if rc != 0:
        raise GlsError(lib().gls_last_error().decode())


def _stream():
    """torch's current stream on the current device, as the C ABI's stream
    argument.  torch._C._cuda_getCurrentRawStream returns the handle without
    building a Stream object (3.0 us per call on the box for the public
    form, profiles/r06/explore/host_overhead.txt); the public form where it
    is absent."""
    import torch
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        return C.c_void_p(raw(torch.cuda.current_device()))
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr())


def _vptr(v):
    """Device tensor or host numpy array (GLS_MEM_HOST layouts)."""
    if isinstance(v, np.ndarray):
        assert v.flags["C_CONTIGUOUS"]
        return C.c_void_p(v.ctypes.data)
    return _ptr(v)


def discover_bricks(mesh_or_cells, dim=None, degree=None):
    """gls_discover_bricks: (shape, perm) for a cell list in any order (host
    only).  Accepts a mesh (cell_nodes, dim, degree) or a cell_nodes array."""
    if dim is None:
        cn, dim, degree = mesh_or_cells.cell_nodes, mesh_or_cells.dim, mesh_or_cells.degree
    else:
        cn = mesh_or_cells
    cn = np.ascontiguousarray(cn, dtype=np.uint32)
    shape = (C.c_int * 3)()
    perm = np.empty(cn.shape[0], dtype=np.int64)
    _check(lib().gls_discover_bricks(int(dim), int(degree), cn.shape[0], cn.ctypes.data, shape,
                                     perm.ctypes.data))
    return tuple(shape), perm


class NavierStokesOperator:
    """Mirror of NavierStokesOperator<dim, Number> (operator_ns.h:17-189) over
    the HIP C-ABI.  precision: "f64" (fine level, Number=double) or "f32"
    (MG levels, MGNumber=float, config.h:6-7)."""

    def __init__(self, mesh, cmask, precision="f64", cells=None, n_owned_nodes=None,
                 brick=None, outflow=None):
        import torch
        if not torch.cuda.is_available():
            raise GlsError("NavierStokesOperator needs a GPU (no CPU fallback by design)")
        self.mesh = mesh
        self.dim = mesh.dim
        self.degree = mesh.degree
        self.prec = GLS_F64 if precision in ("f64", "double", GLS_F64) else GLS_F32
        self.dtype = torch.float64 if self.prec == GLS_F64 else torch.float32
        cell_nodes = mesh.cell_nodes if cells is None else mesh.cell_nodes[cells]
        meas, hmin = mesh.cell_measure()
        if cells is not None:
            meas, hmin = meas[cells], hmin[cells]
        self._keep = [np.ascontiguousarray(cell_nodes, dtype=np.uint32),
                      np.ascontiguousarray(mesh.coords, dtype=np.float64),
                      np.ascontiguousarray(cmask, dtype=np.uint8),
                      np.ascontiguousarray(meas), np.ascontiguousarray(hmin)]
        k = self._keep
        self.n_cells = k[0].shape[0]
        if brick is None:
            brick = mesh.brick() if cells is None else (0, 0, 0)
        elif brick == "auto":  # any cell order: bricks discovered by the library
            brick = (-1, -1, -1)
        self.brick = tuple(brick)
        d = OpDesc(self.dim, self.degree, self.prec, self.n_cells, mesh.n_nodes,
                   mesh.n_nodes if n_owned_nodes is None else n_owned_nodes,
                   k[0].ctypes.data, k[1].ctypes.data, k[2].ctypes.data, k[3].ctypes.data,
                   k[4].ctypes.data, (C.c_int * 3)(*self.brick))
        if outflow is not None:
            # (cells, face_no, kind): the weak outflow faces (all_outflow_bcs_*,
            # operator_ns.cc:79-95); kind "cut" / "nitsche" or per face 1 / 2
            fc, fn, kind = outflow
            fc = np.ascontiguousarray(fc, dtype=np.int64)
            fn = np.ascontiguousarray(fn, dtype=np.int32)
            if isinstance(kind, str):
                kind = np.full(len(fc), OUTFLOW_KIND[kind], dtype=np.int32)
            kind = np.ascontiguousarray(kind, dtype=np.int32)
            self._keep += [fc, fn, kind]
            d.n_outflow_faces = len(fc)
            d.outflow_cells, d.outflow_face_no, d.outflow_kind = (
                fc.ctypes.data, fn.ctypes.data, kind.ctypes.data)
        mp = getattr(mesh, "mapping_points", None)
        mapping = mp() if callable(mp) else None
        if mapping is not None:
            # MappingQ of the parent (FE_Q_iso_Q1 level): per-cell support points
            mdeg, pts = mapping
            pts = np.ascontiguousarray(pts if cells is None else pts[cells], dtype=np.float64)
            self._keep.append(pts)
            d.mapping_degree, d.mapping_points = int(mdeg), pts.ctypes.data
        h = C.c_void_p()
        _check(lib().gls_op_create(C.byref(d), C.byref(h)))
        self.h = h
        self.n_dofs = lib().gls_op_m(h)
        dims = (C.c_int * 3)()
        _check(lib().gls_op_brick_shape(h, dims))
        self.brick_shape = tuple(dims)  # what runs: (0, 0, 0) = per-cell kernel

    def extract_constant_modes(self):
        """NavierStokesOperator::extract_constant_modes (operator_ns.cc:
        175-193, DoFTools::extract_constant_modes over all dim+1 components):
        one boolean dof mask per component, node-major numbering (the AMG
        near-null space a Trilinos coarse solver takes)."""
        nc = self.dim + 1
        comp = np.arange(self.n_dofs) % nc
        return [comp == c for c in range(nc)]

    @property
    def n_outflow_faces(self):
        n, q = C.c_int64(), C.c_int()
        _check(lib().gls_op_n_outflow_faces(self.h, C.byref(n), C.byref(q)))
        return n.value, q.value

    def outflow_face_points(self):
        """[face][point][dim] face quadrature points (gls_op_outflow_face_points)."""
        n, q = self.n_outflow_faces
        x = np.empty((n, q, self.dim))
        _check(lib().gls_op_outflow_face_points(self.h, x.ctypes.data))
        return x

    def set_outflow_target(self, target, stream=None):
        """Nitsche target velocity at the face points, [face][point][dim]
        (face_target_velocity, operator_ns.cc:478-521)."""
        n, q = self.n_outflow_faces
        t = np.ascontiguousarray(target, dtype=np.float64)
        if t.size != n * q * self.dim:
            raise GlsError("set_outflow_target: expected [faces][points][dim]")
        _check(lib().gls_op_set_outflow_target(self.h, t.ctypes.data, stream))

    def element_matrices(self):
        """[cell][row i][col j] element matrices (gls_op_element_matrices;
        local dof = point * (dim+1) + component)."""
        nd = (self.degree + 1) ** self.dim * (self.dim + 1)
        out = np.empty((self.n_cells, nd, nd))
        _check(lib().gls_op_element_matrices(self.h, out.ctypes.data))
        return np.ascontiguousarray(out.transpose(0, 2, 1))

    def system_matrix(self):
        """OperatorBase::get_system_matrix as a scipy CSR matrix over the
        node-major dofs (gls_op_system_matrix)."""
        import scipy.sparse as sp
        nnz = C.c_int64()
        _check(lib().gls_op_system_matrix(self.h, C.byref(nnz), None, None, None))
        rp = np.empty(self.n_dofs + 1, dtype=np.int64)
        cols = np.empty(nnz.value, dtype=np.int64)
        vals = np.empty(nnz.value)
        _check(lib().gls_op_system_matrix(self.h, C.byref(nnz), rp.ctypes.data, cols.ctypes.data,
                                          vals.ctypes.data))
        return sp.csr_matrix((vals, cols, rp), shape=(self.n_dofs, self.n_dofs))

    def cell_permutation(self):
        """perm[internal cell] = caller cell (identity unless bricks were
        discovered)."""
        p = np.empty(self.n_cells, dtype=np.int64)
        _check(lib().gls_op_cell_permutation(self.h, p.ctypes.data))
        return p

    def sweep_stats(self):
        """(resident smoothing launches, slot waits that hit their spin
        bound) on this multigrid level (gls_op_sweep_stats)."""
        n, c = C.c_uint64(0), C.c_uint64(0)
        _check(lib().gls_op_sweep_stats(self.h, C.byref(n), C.byref(c)))
        return int(n.value), int(c.value)

    def set_sweep_spin_bound(self, polls):
        """Polls of a neighbour's slot before a resident sweep's wait gives
        up (gls_op_set_sweep_spin_bound; 0 forces the stall path: tests)."""
        _check(lib().gls_op_set_sweep_spin_bound(self.h, int(polls)))

    def __del__(self):
        try:
            if self.h:
                lib().gls_op_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # --- OperatorBase-like API
    def m(self):
        return self.n_dofs

    def set_parameters(self, nu, c1=1.0, c2=1.0, theta=1.0, w0=0.0, dt=1.0, order=0,
                       increment_form=True, consider_time_derivative=False,
                       cell_wise_stabilization=False, deterministic=False):
        """deterministic: GLS_DETERMINISTIC (not a reference parameter) --
        bitwise reproducible results run to run (ordered lattice
        accumulation, colour-by-colour diagonal and restriction), slower"""
        flags = ((GLS_INCREMENT_FORM if increment_form else 0)
                 | (GLS_CONSIDER_TIME_DERIVATIVE if consider_time_derivative else 0)
                 | (GLS_CELL_WISE_STAB if cell_wise_stabilization else 0)
                 | (GLS_DETERMINISTIC if deterministic else 0))
        self.params = OpParams(nu, c1, c2, theta, w0, dt, order, flags)
        _check(lib().gls_op_set_parameters(self.h, C.byref(self.params)))

    def initialize_dof_vector(self):
        import torch
        return torch.zeros(self.n_dofs, dtype=self.dtype, device="cuda")

    def _dev(self, v):
        import torch
        if isinstance(v, np.ndarray):
            v = torch.from_numpy(v)
        return v.to(device="cuda", dtype=self.dtype).contiguous()

    def _arg(self, v):
        """A vector argument in the current layout: numpy (host layout) or a
        device tensor."""
        if getattr(self, "_memory", "device") == "host":
            return np.ascontiguousarray(v, dtype=np.float64 if self.prec == GLS_F64
                                        else np.float32)
        return self._dev(v)

    def set_linearization_point(self, vec):
        v = self._arg(vec)
        _check(lib().gls_op_set_linearization_point(self.h, _vptr(v), _stream()))

    def set_previous_solution(self, history, weights):
        hs = [self._arg(h) for h in history]
        ptrs = (C.c_void_p * len(hs))(*[_vptr(h).value for h in hs])
        w = np.ascontiguousarray(weights, dtype=np.float64)
        _check(lib().gls_op_set_previous_solution(self.h, C.cast(ptrs, C.c_void_p), len(hs),
                                                  w.ctypes.data, _stream()))
        self._hist_keep = hs

    def vmult(self, dst, src):
        _check(lib().gls_op_vmult(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def Tvmult(self, dst, src):
        """OperatorBase::Tvmult forwards to vmult (operator_base.cc:12-18)."""
        self.vmult(dst, src)

    def vmult_interface_down(self, dst, src):
        """OperatorBase::vmult_interface_down (operator_ns.cc:734-753): on a
        globally refined level (no refinement-edge dofs) the vmult."""
        _check(lib().gls_op_vmult_interface_down(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def vmult_interface_up(self, dst, src):
        """OperatorBase::vmult_interface_up (operator_ns.cc:755-787): dst = 0
        without refinement-edge dofs (has_edge_constrained_indices false)."""
        _check(lib().gls_op_vmult_interface_up(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def invalidate_system(self):
        """OperatorBase::invalidate_system (operator_ns.cc:229-232): the
        reference drops its cached system matrix; system_matrix() here is
        assembled on every call, so there is nothing to drop."""

    def get_constraints(self):
        """The homogeneous constraints the operator resolves
        (get_constraints, operator_ns.cc:157-160): per node the constrained
        component bits, node-major."""
        return np.asarray(self._keep[2])

    def vmult_init(self, dst, src):
        _check(lib().gls_op_vmult_init(self.h, _ptr(dst), _ptr(src), _stream()))

    def apply_identity_rows(self, dst, src):
        _check(lib().gls_op_apply_identity_rows(self.h, _ptr(dst), _ptr(src), _stream()))

    def vmult_cells(self, dst, src, begin, end):
        _check(lib().gls_op_vmult_cells(self.h, _ptr(dst), _ptr(src), int(begin), int(end),
                                        _stream()))

    def evaluate_residual(self, dst, src):
        """operator_ns.cc:648-682: distribute the inhomogeneous constraints
        on a copy of src, residual cell loop, set_zero, *= -1."""
        _check(lib().gls_op_evaluate_residual(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def evaluate_residual_plain(self, dst, src):
        """The same on src as it is (no distribute)."""
        _check(lib().gls_op_evaluate_residual_plain(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def evaluate_rhs(self, dst):
        """operator_ns.cc:622-646: residual of the zero vector with the
        inhomogeneous constraints distributed."""
        _check(lib().gls_op_evaluate_rhs(self.h, _vptr(dst), _stream()))
        return dst

    def set_constraint_values(self, values):
        """constraints_inhomogeneous (main.cc:879-891): a dof vector whose
        constrained components hold the Dirichlet values (None: all zero)."""
        if values is None:
            _check(lib().gls_op_set_constraint_values(self.h, None, _stream()))
            return
        v = self._dev(values)
        _check(lib().gls_op_set_constraint_values(self.h, _ptr(v), _stream()))
        self._inhom_keep = v

    def compute_inverse_diagonal(self, diag):
        _check(lib().gls_op_compute_inverse_diagonal(self.h, _vptr(diag), _stream()))
        return diag

    def compute_diagonal(self, diag):
        """Assembled (not inverted) diagonal: the rank-local half of a
        partitioned compute_inverse_diagonal."""
        _check(lib().gls_op_compute_diagonal(self.h, _ptr(diag), _stream()))
        return diag

    def invert_diagonal(self, diag):
        _check(lib().gls_op_invert_diagonal(self.h, _ptr(diag), _stream()))
        return diag

    def get_max_u(self, vec):
        """OperatorBase::get_max_u (operator_ns.cc:530-568): max |u(x_q)|."""
        out = C.c_double()
        _check(lib().gls_op_get_max_u(self.h, _vptr(vec), C.byref(out), _stream()))
        return out.value

    def set_vector_layout(self, memory="device", dof_map=None):
        """Caller vector layout (gls_op_set_vector_layout): memory "host"
        (numpy arrays, staged) or "device" (torch tensors); dof_map[i] = the
        node-major dof of caller dof i (deal.II numbering), or None."""
        m = np.ascontiguousarray(dof_map, dtype=np.int64) if dof_map is not None else None
        _check(lib().gls_op_set_vector_layout(self.h, GLS_MEM_HOST if memory == "host"
                                              else GLS_MEM_DEVICE,
                                              None if m is None else m.ctypes.data))
        self._map_keep = m
        self._memory = memory

    def download_tables(self):
        nq = (self.degree + 1) ** self.dim
        nf = 2 + 3 * self.dim + self.dim ** 2
        t = np.empty((self.n_cells, nq, nf))
        cw = np.empty((self.n_cells, 2))
        _check(lib().gls_op_download_tables(self.h, t.ctypes.data, cw.ctypes.data))
        return t, cw

    def upload_tables(self, tables, cellwise=None):
        t = np.ascontiguousarray(tables, dtype=np.float64)
        cw = None if cellwise is None else np.ascontiguousarray(cellwise, dtype=np.float64)
        _check(lib().gls_op_upload_tables(self.h, t.ctypes.data,
                                          None if cw is None else cw.ctypes.data))

    def geometry_counts(self):
        g, c = C.c_int64(), C.c_int64()
        _check(lib().gls_op_geometry_counts(self.h, C.byref(g), C.byref(c)))
        return g.value, c.value

    def vmult_bytes(self):
        return lib().gls_op_vmult_bytes(self.h)


def dist_unique_id():
    """128-byte RCCL unique id (one rank creates it, all ranks use it)."""
    b = (C.c_char * 128)()
    _check(lib().gls_dist_unique_id(C.cast(b, C.c_void_p)))
    return bytes(b)


class PartitionedOperator:
    """The rank-local half of a partitioned NavierStokesOperator: ghost
    import / compress(add) over RCCL (nccl_id given) or inside an in-process
    group of ranks on one device (nccl_id None, `group` = a member created
    before).  op: the rank-local NavierStokesOperator; recv blocks: per peer
    the [begin, begin + count) local ghost nodes it owns; send_nodes: per peer
    the owned local nodes that are ghosts there, in the peer's ghost order."""

    def __init__(self, op, rank, world, peers, send_nodes, recv_blocks, nccl_id=None,
                 group=None):
        self.op = op
        peers = [int(q) for q in peers]
        self._keep = [np.ascontiguousarray(peers, dtype=np.int32),
                      np.ascontiguousarray([len(send_nodes[q]) for q in peers], dtype=np.int64),
                      np.ascontiguousarray(np.concatenate([np.asarray(send_nodes[q], np.int64)
                                                           for q in peers])
                                           if peers else np.zeros(0), dtype=np.uint32),
                      np.ascontiguousarray([recv_blocks[q][0] for q in peers], dtype=np.int64),
                      np.ascontiguousarray([recv_blocks[q][1] for q in peers], dtype=np.int64)]
        k = self._keep
        idb = None
        if nccl_id is not None:
            idb = (C.c_char * 128).from_buffer_copy(bytes(nccl_id))
            self._keep.append(idb)
        d = DistDesc(rank, world, None if idb is None else C.cast(idb, C.c_void_p),
                     None if group is None else group.h, len(peers), k[0].ctypes.data,
                     k[1].ctypes.data, k[2].ctypes.data, k[3].ctypes.data, k[4].ctypes.data)
        h = C.c_void_p()
        _check(lib().gls_dist_create(op.h, C.byref(d), C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().gls_dist_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def vmult(self, dst, src):
        _check(lib().gls_dist_vmult(self.h, _ptr(dst), _ptr(src), _stream()))
        return dst

    def update_ghost_values(self, vec):
        _check(lib().gls_dist_update_ghost_values(self.h, _ptr(vec), _stream()))

    def compress_add(self, vec):
        _check(lib().gls_dist_compress_add(self.h, _ptr(vec), _stream()))

    def get_max_u(self, vec):
        """get_max_u of the partitioned operator: ghost import, local max,
        RCCL all-reduce max (operator_ns.cc:540-567)."""
        out = C.c_double()
        _check(lib().gls_dist_get_max_u(self.h, _ptr(vec), C.byref(out), _stream()))
        return out.value

    def interior_bricks(self):
        a, b = C.c_int64(), C.c_int64()
        _check(lib().gls_dist_interior_bricks(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    @staticmethod
    def vmult_group(members, dsts, srcs):
        n = len(members)
        hs = (C.c_void_p * n)(*[m.h.value for m in members])
        ds = (C.c_void_p * n)(*[d.data_ptr() for d in dsts])
        ss = (C.c_void_p * n)(*[s.data_ptr() for s in srcs])
        _check(lib().gls_dist_vmult_group(C.cast(hs, C.c_void_p), C.cast(ds, C.c_void_p),
                                          C.cast(ss, C.c_void_p), n, _stream()))
        return dsts


class DistMGDesc(C.Structure):
    _fields_ = [("mg", MGDesc), ("child", C.c_void_p), ("owned_global_nodes", C.c_void_p),
                ("n_global_nodes", C.c_void_p), ("coarse_global", C.c_void_p),
                ("coarse_local_global", C.c_void_p), ("n_redundant_levels", C.c_int),
                ("redundant_ops", C.c_void_p), ("redundant_child", C.c_void_p)]


def _handles(objs):
    n = len(objs)
    return (C.c_void_p * n)(*[o.h.value for o in objs]), n


def _ptrs(ts):
    return (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


class PartitionedMultigrid:
    """The rank-local handle of the native partitioned multigrid
    (gls_dist_mg_*, csrc/dist_mg.hip): PreconditionerGMG over partitioned
    level operators (PartitionedOperator handles of one rank, coarse to
    fine).  child[l] (l >= 1): rank-local child lattice with the global-first
    NOT_OWNER bits; owned_global_nodes[l]: global ids of the owned nodes;
    coarse_global (direct coarse solve): a NavierStokesOperator on the whole
    coarse mesh with coarse_l2g (level-0 local node -> global node).
    Agglomeration (glsDistMGDesc n_redundant_levels): redundant_ops, the
    global NavierStokesOperators of the levels below level 0 (coarsest
    first), and redundant_child[l] (l = 1 .. len(redundant_ops); entry 0
    unused) the global child lattices up to coarse_global's mesh: those
    levels run single-domain on every rank.  The team methods take every
    handle this process drives: [self] for an RCCL rank, all members of an
    in-process group in rank order (tests)."""

    def __init__(self, levels, child, owned_global_nodes, n_global_nodes,
                 smoothing_n_iterations=5, smoothing_eig_n_iterations=20, smoothing_range=20.0,
                 coarse_n_iterations=10, outer_precision="f64", compute_evs_n_levels=0,
                 coarse_global=None, coarse_l2g=None, redundant_ops=None, redundant_child=None):
        n = len(levels)
        outer = GLS_F64 if outer_precision in ("f64", GLS_F64) else GLS_F32
        md = MGDesc(n, smoothing_n_iterations, smoothing_eig_n_iterations, smoothing_range,
                    coarse_n_iterations, outer, compute_evs_n_levels, 0, 1e-4, 10000)
        self._keep = [None] + [np.ascontiguousarray(c, dtype=np.uint32) for c in child[1:]]
        self._own = [np.ascontiguousarray(g, dtype=np.int64) for g in owned_global_nodes]
        self._ng = np.ascontiguousarray(n_global_nodes, dtype=np.int64)
        chp = (C.c_void_p * n)(*([None] + [c.ctypes.data for c in self._keep[1:]]))
        ogp = (C.c_void_p * n)(*[g.ctypes.data for g in self._own])
        self._l2g = None if coarse_l2g is None else np.ascontiguousarray(coarse_l2g, np.int64)
        self.coarse_global = coarse_global
        nr = len(redundant_ops) if redundant_ops else 0
        self.redundant_ops = list(redundant_ops or [])
        self._rch = [None] + [np.ascontiguousarray(c, dtype=np.uint32)
                              for c in (redundant_child or [None])[1:]]
        rop = (C.c_void_p * max(nr, 1))(*[o.h.value for o in self.redundant_ops])
        rch = (C.c_void_p * (nr + 1))(*([None] + [c.ctypes.data for c in self._rch[1:]]))
        d = DistMGDesc(md, C.cast(chp, C.c_void_p), C.cast(ogp, C.c_void_p),
                       self._ng.ctypes.data,
                       None if coarse_global is None else coarse_global.h,
                       None if self._l2g is None else self._l2g.ctypes.data, nr,
                       C.cast(rop, C.c_void_p) if nr else None,
                       C.cast(rch, C.c_void_p) if nr else None)
        lv = (C.c_void_p * n)(*[L.h.value for L in levels])
        h = C.c_void_p()
        _check(lib().gls_dist_mg_create(C.byref(d), C.cast(lv, C.c_void_p), C.byref(h)))
        self.h = h
        self._ptr_keep = (chp, ogp, lv, rop, rch)
        self.levels = levels

    def __del__(self):
        try:
            if self.h:
                lib().gls_dist_mg_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def relaxation(self, level):
        w, lam = C.c_double(), C.c_double()
        _check(lib().gls_dist_mg_get_relaxation(self.h, level, C.byref(w), C.byref(lam)))
        return w.value, lam.value

    @staticmethod
    def set_linearization_point(team, u_fine, hist_fine=None, weights=None):
        hs, n = _handles(team)
        us = _ptrs(u_fine)
        nh = 0 if not hist_fine else len(hist_fine[0])
        hrows = [_ptrs(h) for h in hist_fine] if nh else []
        hp = (C.c_void_p * n)(*[C.cast(r, C.c_void_p).value for r in hrows]) if nh else None
        w = None
        if weights is not None:
            w = np.ascontiguousarray(weights, dtype=np.float64)
        _check(lib().gls_dist_mg_set_linearization_point(
            C.cast(hs, C.c_void_p), n, C.cast(us, C.c_void_p),
            None if hp is None else C.cast(hp, C.c_void_p), nh,
            None if w is None else w.ctypes.data, _stream()))

    @staticmethod
    def setup(team):
        hs, n = _handles(team)
        _check(lib().gls_dist_mg_setup(C.cast(hs, C.c_void_p), n, _stream()))

    @staticmethod
    def vcycle(team, dsts, srcs):
        hs, n = _handles(team)
        _check(lib().gls_dist_mg_vcycle(C.cast(hs, C.c_void_p), n, C.cast(_ptrs(dsts), C.c_void_p),
                                        C.cast(_ptrs(srcs), C.c_void_p), _stream()))
        return dsts


def dist_gmres_solve(ops, mgs, xs, bs, n_max_iterations=10000, absolute_tolerance=1e-12,
                     relative_tolerance=1e-8, max_n_tmp_vectors=30):
    """gls_dist_gmres_solve: LinearSolverGMRES::solve on rank-local vectors of
    the FP64 partitioned operator (PartitionedOperator handles of the team),
    preconditioned by the native partitioned multigrid (or identity, mgs
    None).  Returns the result dict; raises GlsError on no convergence."""
    hs, n = _handles(ops)
    ms = None if mgs is None else _handles(mgs)[0]
    desc = GMRESDesc(max_n_tmp_vectors, n_max_iterations, absolute_tolerance, relative_tolerance)
    res = GMRESResult()
    rc = lib().gls_dist_gmres_solve(C.cast(hs, C.c_void_p),
                                    None if ms is None else C.cast(ms, C.c_void_p), n,
                                    C.byref(desc), C.cast(_ptrs(xs), C.c_void_p),
                                    C.cast(_ptrs(bs), C.c_void_p), C.byref(res), _stream())
    out = {f: getattr(res, f) for f, _ in GMRESResult._fields_}
    _check(rc)
    return out


class AMG:
    """TrilinosWrappers::PreconditionAMG over the C-ABI (gls_amg_*): built
    from a scipy CSR matrix (initialize), vmult = one V-cycle on device FP64
    vectors.  The substitute for Trilinos ML (csrc/amg.hip)."""

    def __init__(self, matrix, **params):
        import torch
        if not torch.cuda.is_available():
            raise GlsError("AMG needs a GPU (no CPU fallback by design)")
        A = matrix.tocsr()
        A.sort_indices()
        rp = np.ascontiguousarray(A.indptr, dtype=np.int64)
        ci = np.ascontiguousarray(A.indices, dtype=np.int64)
        va = np.ascontiguousarray(A.data, dtype=np.float64)
        self.prm = amg_params(**params)
        h = C.c_void_p()
        _check(lib().gls_amg_create(A.shape[0], rp.ctypes.data, ci.ctypes.data, va.ctypes.data,
                                    C.byref(self.prm), C.byref(h)))
        self.h = h
        self.n = A.shape[0]

    @staticmethod
    def _info_of(h):
        nl = C.c_int()
        _check(lib().gls_amg_info(h, C.byref(nl), None, None, None))
        sizes = np.zeros(nl.value, dtype=np.int64)
        nnz = np.zeros(nl.value, dtype=np.int64)
        lam = np.zeros(nl.value)
        _check(lib().gls_amg_info(h, C.byref(nl), sizes.ctypes.data, nnz.ctypes.data,
                                  lam.ctypes.data))
        return {"levels": nl.value, "sizes": sizes.tolist(), "nnz": nnz.tolist(),
                "lambda": lam.tolist()}

    def info(self):
        return self._info_of(self.h)

    def level_matrix(self, level, which="A"):
        """the device hierarchy's A / P / R of a level as scipy CSR"""
        import scipy.sparse as sp
        w = {"A": 0, "P": 1, "R": 2}[which]
        n, nnz = C.c_int64(), C.c_int64()
        _check(lib().gls_amg_level_matrix(self.h, level, w, C.byref(n), C.byref(nnz), None, None,
                                          None))
        rp = np.zeros(n.value + 1, dtype=np.int32)
        ci = np.zeros(nnz.value, dtype=np.int32)
        va = np.zeros(nnz.value)
        _check(lib().gls_amg_level_matrix(self.h, level, w, C.byref(n), C.byref(nnz),
                                          rp.ctypes.data, ci.ctypes.data, va.ctypes.data))
        m = int(ci.max()) + 1 if nnz.value else 0
        return sp.csr_matrix((va, ci, rp), shape=(n.value, max(m, 1)))

    def vmult(self, dst, src):
        _check(lib().gls_amg_vmult(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def __del__(self):
        try:
            if self.h:
                lib().gls_amg_destroy(self.h)
                self.h = None
        except Exception:
            pass


class Multigrid:
    """PreconditionerGMG (multigrid.h:61-141) over the C-ABI: level operators
    (MGNumber = float by default), damped-Jacobi relaxation smoother with a
    power-iteration relaxation factor, MGTwoLevelTransfer, V-cycle."""

    def __init__(self, level_ops, child_lattices, smoothing_n_iterations=5,
                 smoothing_eig_n_iterations=20, smoothing_range=20.0, coarse_n_iterations=20,
                 outer_precision="f64", compute_evs_n_levels=0, coarse_iterate=False,
                 coarse_reltol=1e-4, coarse_maxiter=10000, coarse_amg=None):
        self.ops = list(level_ops)
        self._child = [None] + [np.ascontiguousarray(c, dtype=np.uint32)
                                for c in child_lattices]
        n = len(self.ops)
        arr = (C.c_void_p * n)(*[op.h.value for op in self.ops])
        ch = (C.c_void_p * n)(*[0 if c is None else c.ctypes.data for c in self._child])
        outer = GLS_F64 if outer_precision in ("f64", GLS_F64) else GLS_F32
        self.desc = MGDesc(n, smoothing_n_iterations, smoothing_eig_n_iterations,
                           smoothing_range, coarse_n_iterations, outer, compute_evs_n_levels,
                           int(bool(coarse_iterate)), coarse_reltol, coarse_maxiter)
        if coarse_amg is not None:
            # "gmg coarse grid solver": "AMG": a dict of amg_params() keywords
            # or an AMGParams
            self.desc.coarse_amg = 1
            self.desc.amg = (coarse_amg if isinstance(coarse_amg, AMGParams)
                             else amg_params(**coarse_amg))
        self.outer_dtype = None
        h = C.c_void_p()
        _check(lib().gls_mg_create(C.byref(self.desc), C.cast(arr, C.c_void_p),
                                   C.cast(ch, C.c_void_p), C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().gls_mg_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def setup(self):
        _check(lib().gls_mg_setup(self.h, _stream()))

    def coarse_statistics(self):
        """(GMRES iterations, converged) of the last coarse solve
        (coarse_iterate=True)."""
        it, cv = C.c_int(), C.c_int()
        _check(lib().gls_mg_coarse_statistics(self.h, C.byref(it), C.byref(cv)))
        return it.value, bool(cv.value)

    def coarse_setup_times(self):
        """{assembly_ms, getrf_ms, inverse_ms, colors} of the last dense-coarse
        setup (coarse_n_iterations=-1); inverse_ms: the inverse from the LU
        factors (trtri + trsm by default, GLS_COARSE_REFERENCE=getrs|getri)."""
        ms = (C.c_double * 3)()
        nc = C.c_int()
        _check(lib().gls_mg_coarse_setup_times(self.h, ms, C.byref(nc)))
        return {"assembly_ms": ms[0], "getrf_ms": ms[1], "inverse_ms": ms[2],
                "colors": nc.value}

    def coarse_amg(self):
        """(AMG info dict, setup ms) of the coarse AMG (coarse_amg given), or
        None before setup."""
        h, ms = C.c_void_p(), C.c_double()
        _check(lib().gls_mg_coarse_amg(self.h, C.byref(h), C.byref(ms)))
        if not h.value:
            return None
        return AMG._info_of(h), ms.value

    def relaxation(self, level):
        w, lam = C.c_double(), C.c_double()
        _check(lib().gls_mg_get_relaxation(self.h, level, C.byref(w), C.byref(lam)))
        return w.value, lam.value

    def vcycle(self, dst, src):
        _check(lib().gls_mg_vcycle(self.h, _vptr(dst), _vptr(src), _stream()))
        return dst

    def set_vector_layout(self, memory="device", dof_map=None):
        m = np.ascontiguousarray(dof_map, dtype=np.int64) if dof_map is not None else None
        _check(lib().gls_mg_set_vector_layout(self.h, GLS_MEM_HOST if memory == "host"
                                              else GLS_MEM_DEVICE,
                                              None if m is None else m.ctypes.data))
        self._map_keep = m

    def prolongate_add(self, level, dst_fine, src_coarse):
        _check(lib().gls_mg_prolongate_add(self.h, level, _ptr(dst_fine), _ptr(src_coarse),
                                           _stream()))

    def restrict_add(self, level, dst_coarse, src_fine):
        _check(lib().gls_mg_restrict_add(self.h, level, _ptr(dst_coarse), _ptr(src_fine),
                                         _stream()))

    def interpolate(self, level, dst_coarse, src_fine):
        _check(lib().gls_mg_interpolate(self.h, level, _ptr(dst_coarse), _ptr(src_fine),
                                        _stream()))

    def relax(self, level, x, b, ax, inv_diag, omega, zero_start):
        """x = omega d b (zero_start) or x += omega d (b - ax): one damped
        Jacobi update (the distributed smoother's elementwise half)."""
        _check(lib().gls_mg_relax(self.h, level, _ptr(x), _ptr(b),
                                  None if ax is None else _ptr(ax), _ptr(inv_diag),
                                  float(omega), int(zero_start), _stream()))

    def smooth(self, level, x, b, zero_initial_guess=True):
        _check(lib().gls_mg_smooth(self.h, level, _ptr(x), _ptr(b), int(zero_initial_guess),
                                   _stream()))


def build_gmg(meshes, cmasks, params, u_star_fine, history_fine=None, weights=None,
              precision="f32", coarse_iso_q1=False, outflow=None, **mg_kwargs):
    """Level operators + transfers for a mesh hierarchy (coarse -> fine), the
    linearization point / history interpolated down level by level
    (interpolate_to_mg, main.cc:772-803, 815-832).  coarse_iso_q1: the
    coarsest level with FE_Q_iso_Q1 (glsmesh.IsoQ1Mesh, main.cc:436-446).
    outflow: None, or (kind, boundary id): every level operator gets its
    mesh's outflow faces (the level operators take the outflow sets too,
    main.cc:520-527).  Returns (mg, level_ops)."""
    import torch
    if coarse_iso_q1:
        import glsmesh
        meshes = [glsmesh.IsoQ1Mesh(meshes[0])] + list(meshes[1:])
    ops = []
    for m, cm in zip(meshes, cmasks):
        of = None
        if outflow is not None:
            import glsmesh
            fc, fn = glsmesh.boundary_faces(m, outflow[1])
            of = (fc, fn, outflow[0])
        op = NavierStokesOperator(m, cm, precision, outflow=of)
        op.set_parameters(**params)
        ops.append(op)
    child = [meshes[l - 1].child_lattice(meshes[l]) for l in range(1, len(meshes))]
    mg = Multigrid(ops, child, **mg_kwargs)
    vecs = [ops[-1]._dev(u_star_fine)]
    hists = [[ops[-1]._dev(h) for h in history_fine]] if history_fine is not None else None
    for l in range(len(ops) - 1, 0, -1):
        v = ops[l - 1].initialize_dof_vector()
        mg.interpolate(l, v, vecs[0])
        vecs.insert(0, v)
        if hists is not None:
            hl = []
            for h in hists[0]:
                t = ops[l - 1].initialize_dof_vector()
                mg.interpolate(l, t, h)
                hl.append(t)
            hists.insert(0, hl)
    for l, op in enumerate(ops):
        op.set_linearization_point(vecs[l])
        if hists is not None and params.get("order", 0) > 0:
            op.set_previous_solution(hists[l], weights)
    torch.cuda.synchronize()
    mg.setup()
    return mg, ops


class LinearSolverGMRES:
    """LinearSolverGMRES (solver_l.h:60-82, solver_l.cc:26-74) over the
    device-resident gls_gmres_solve: right-preconditioned GMRES with 30
    temporary vectors, tolerance max(relative * |b|, absolute), dst zeroed
    first.  `preconditioner` is a Multigrid (one V-cycle per application,
    PreconditionerGMG::vmult) or None (identity).  solve() raises GlsError on
    no convergence (deal.II's SolverControl::NoConvergence); the statistics of
    the last solve are in .last (n_iterations = SolverControl::last_step())."""

    def __init__(self, op, preconditioner=None, n_max_iterations=10000,
                 absolute_tolerance=1e-12, relative_tolerance=1e-8, max_n_tmp_vectors=30):
        self.op = op
        self.preconditioner = preconditioner
        self.desc = GMRESDesc(max_n_tmp_vectors, n_max_iterations, absolute_tolerance,
                              relative_tolerance)
        self.last = None

    def initialize(self):
        pass  # solver_l.cc:39-43: nothing to do

    def solve(self, dst, src):
        res = GMRESResult()
        mg = self.preconditioner.h if self.preconditioner is not None else None
        rc = lib().gls_gmres_solve(self.op.h, mg, C.byref(self.desc), _vptr(dst), _vptr(src),
                                   C.byref(res), _stream())
        self.last = {f: getattr(res, f) for f, _ in GMRESResult._fields_}
        _check(rc)
        return dst
