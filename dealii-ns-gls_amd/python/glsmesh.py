"""ctypes binding of libglsmesh.so (include/gls_mesh.h) + the deck reader.

Problem setup for the hot path: the refined cylinder / hyper-cube meshes of
the five BASELINE decks, their Q_k node numbering, boundary ids and the
constrained-component masks of the boundary descriptor.  See
include/gls_mesh.h for the reference lines each function restates.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import itertools
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.normpath(os.path.join(_HERE, "..", "lib"))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(LIBDIR, "libglsmesh.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make mesh` (or __graft_entry__.build())")
        L = C.CDLL(path)
        vp = C.c_void_p
        L.gls_mesh_cylinder.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                        C.c_double, C.c_double, C.c_double, C.POINTER(vp)]
        L.gls_mesh_hypercube.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
        L.gls_mesh_from_coarse.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int64, vp, C.c_int64,
                                           vp, C.c_int64, vp, vp, C.POINTER(vp)]
        L.gls_mesh_destroy.argtypes = [vp]
        for name in ("gls_mesh_dim", "gls_mesh_degree"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = C.c_int
        for name in ("gls_mesh_n_cells", "gls_mesh_n_nodes", "gls_mesh_n_coarse_cells"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = C.c_int64
        for name in ("gls_mesh_cell_nodes", "gls_mesh_node_coords", "gls_mesh_node_boundary",
                     "gls_mesh_cell_coarse"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = vp
        L.gls_mesh_constraint_mask.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, vp]
        L.gls_mesh_child_lattice.argtypes = [vp, vp, vp]
        L.gls_mesh_cell_measure.argtypes = [vp, vp, vp]
        L.gls_mesh_brick.argtypes = [vp, vp]
        L.gls_mesh_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(lib().gls_mesh_last_error().decode())


def _view(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    ct = np.ctypeslib.as_ctypes_type(dtype)
    arr = np.ctypeslib.as_array((ct * n).from_address(ptr))
    return arr.copy()


class Mesh:
    """A refined mesh with Q_k node numbering (dof = node*(dim+1)+comp)."""

    def __init__(self, handle, kind, params):
        self._h = C.c_void_p(handle)
        self.kind = kind
        self.params = params
        L = lib()
        self.dim = L.gls_mesh_dim(self._h)
        self.degree = L.gls_mesh_degree(self.h)
        self.n_cells = L.gls_mesh_n_cells(self._h)
        self.n_nodes = L.gls_mesh_n_nodes(self._h)
        self.n_coarse_cells = L.gls_mesh_n_coarse_cells(self._h)
        self.nloc = (self.degree + 1) ** self.dim
        self.cell_nodes = _view(L.gls_mesh_cell_nodes(self._h), self.n_cells * self.nloc,
                                np.uint32).reshape(self.n_cells, self.nloc)
        self.coords = _view(L.gls_mesh_node_coords(self._h), self.n_nodes * self.dim,
                            np.float64).reshape(self.n_nodes, self.dim)
        self.node_boundary = _view(L.gls_mesh_node_boundary(self._h), self.n_nodes, np.uint32)
        self.cell_coarse = _view(L.gls_mesh_cell_coarse(self._h), self.n_cells, np.int32)

    @property
    def h(self):
        return self._h

    @property
    def n_dofs(self):
        return self.n_nodes * (self.dim + 1)

    def __del__(self):
        try:
            if self._h:
                lib().gls_mesh_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def constraint_mask(self, vel_ids=(), p_ids=(), slip_ids=()):
        out = np.zeros(self.n_nodes, dtype=np.uint8)
        bits = lambda ids: sum(1 << int(i) for i in ids)
        _check(lib().gls_mesh_constraint_mask(self._h, bits(vel_ids), bits(p_ids),
                                              bits(slip_ids), out.ctypes.data))
        return out

    def brick(self):
        """(bx, by, bz): cells per brick (gls_mesh_brick)."""
        dims = (C.c_int * 3)()
        _check(lib().gls_mesh_brick(self._h, dims))
        return tuple(dims)

    def cell_measure(self):
        meas = np.zeros(self.n_cells)
        hmin = np.zeros(self.n_cells)
        _check(lib().gls_mesh_cell_measure(self._h, meas.ctypes.data, hmin.ctypes.data))
        return meas, hmin

    def child_lattice(self, fine: "Mesh"):
        L = 2 * self.degree + 1
        out = np.zeros((self.n_cells, L ** self.dim), dtype=np.uint32)
        _check(lib().gls_mesh_child_lattice(self._h, fine._h, out.ctypes.data))
        return out


def cylinder(dim, degree, n_ref, length=None, height=0.41, position=None, diameter=0.1,
             shift=0.005):
    """Channel with cylinder (grid_cylinder.h; defaults simulation.cc:210-215)."""
    if length is None:
        length = 2.2 if dim == 2 else 2.5
    if position is None:
        position = 0.2 if dim == 2 else 0.5
    h = C.c_void_p()
    _check(lib().gls_mesh_cylinder(dim, degree, n_ref, length, height, position, diameter,
                                   shift, C.byref(h)))
    return Mesh(h.value, "cylinder", dict(dim=dim, degree=degree, n_ref=n_ref, length=length,
                                          height=height, position=position,
                                          diameter=diameter, shift=shift))


# gmsh hexahedron / quadrangle vertex order -> lexicographic (x fastest)
_GMSH_HEX_LEX = [0, 1, 3, 2, 4, 5, 7, 6]
_GMSH_QUAD_LEX = [0, 1, 3, 2]


def read_msh(path):
    """GridIn::read_msh for gmsh 4.1 ASCII files with linear hexahedra
    (simulation.cc:858-872): vertices, cells (lexicographic vertex order,
    left-handed cells mirrored), boundary quadrilaterals and their physical
    tags (the boundary ids; an entity without one gives 0).  Returns a dict
    of numpy arrays (vertices [nv,3], cells [nc,8], bfaces [nf,4], bids [nf])."""
    with open(path) as f:
        lines = [ln.strip() for ln in f]
    pos = {ln: i for i, ln in enumerate(lines) if ln.startswith("$")}
    fmt = lines[pos["$MeshFormat"] + 1].split()
    if not fmt[0].startswith("4") or fmt[1] != "0":
        raise ValueError(f"{path}: only gmsh 4.x ASCII is supported (got {fmt})")
    # entities -> physical tag
    i = pos["$Entities"] + 1
    counts = [int(x) for x in lines[i].split()]
    i += 1
    phys = {}
    for dim_e, n in enumerate(counts):
        for _ in range(n):
            t = lines[i].split()
            i += 1
            tag = int(t[0])
            k = 4 if dim_e == 0 else 7
            nphys = int(t[k])
            phys[(dim_e, tag)] = abs(int(t[k + 1])) if nphys > 0 else 0
    # nodes
    i = pos["$Nodes"] + 1
    nblocks, nnodes = (int(x) for x in lines[i].split()[:2])
    i += 1
    tags, xyz = [], []
    for _ in range(nblocks):
        _, _, parametric, nb = (int(x) for x in lines[i].split())
        i += 1
        tags.extend(int(lines[i + j]) for j in range(nb))
        i += nb
        for j in range(nb):
            xyz.append([float(x) for x in lines[i + j].split()[:3]])
        i += nb
    index = {t: j for j, t in enumerate(tags)}
    vertices = np.asarray(xyz, dtype=np.float64)
    # elements
    i = pos["$Elements"] + 1
    nblocks = int(lines[i].split()[0])
    i += 1
    cells, bfaces, bids = [], [], []
    for _ in range(nblocks):
        edim, etag, etype, nb = (int(x) for x in lines[i].split())
        i += 1
        for j in range(nb):
            v = [index[int(x)] for x in lines[i + j].split()[1:]]
            if etype == 5:
                cells.append([v[k] for k in _GMSH_HEX_LEX])
            elif etype == 3:
                bfaces.append([v[k] for k in _GMSH_QUAD_LEX])
                bids.append(phys.get((edim, etag), 0))
        i += nb
    cells = np.asarray(cells, dtype=np.int32)
    # mirror left-handed cells (deal.II reorders them to positive measure)
    p = vertices[cells]
    jac = np.einsum("ci,ci->c", np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]),
                    p[:, 4] - p[:, 0])
    neg = jac < 0
    cells[neg] = cells[neg][:, [1, 0, 3, 2, 5, 4, 7, 6]]
    return dict(vertices=vertices, cells=cells, bfaces=np.asarray(bfaces, dtype=np.int32),
                bids=np.asarray(bids, dtype=np.int32))


def from_coarse(coarse, degree, n_ref, kind="coarse"):
    """A refined mesh from a coarse hex mesh (gls_mesh_from_coarse)."""
    v = np.ascontiguousarray(coarse["vertices"], dtype=np.float64)
    c = np.ascontiguousarray(coarse["cells"], dtype=np.int32)
    bf = np.ascontiguousarray(coarse["bfaces"], dtype=np.int32)
    bi = np.ascontiguousarray(coarse["bids"], dtype=np.int32)
    dim = v.shape[1]
    h = C.c_void_p()
    _check(lib().gls_mesh_from_coarse(dim, degree, n_ref, v.shape[0], v.ctypes.data, c.shape[0],
                                      c.ctypes.data, bf.shape[0], bf.ctypes.data, bi.ctypes.data,
                                      C.byref(h)))
    return Mesh(h.value, kind, dict(dim=dim, degree=degree, n_ref=n_ref))


SPHERE_COARSE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data",
                             "sphere_coarse.npz")


def sphere(degree, n_ref, path=None):
    """SimulationSphere::create_triangulation (simulation.cc:858-872): the
    reference's mesh/sphere.msh (or its converted coarse arrays,
    data/sphere_coarse.npz, scripts/convert_msh.py) refined n_ref times."""
    if path is not None and path.endswith(".msh"):
        coarse = read_msh(path)
    else:
        with np.load(path or SPHERE_COARSE) as z:
            coarse = {k: z[k] for k in z.files}
    return from_coarse(coarse, degree, n_ref, "sphere")


def hypercube(dim, degree, n_ref):
    h = C.c_void_p()
    _check(lib().gls_mesh_hypercube(dim, degree, n_ref, C.byref(h)))
    return Mesh(h.value, "hypercube", dict(dim=dim, degree=degree, n_ref=n_ref))


def boundary_faces(mesh, bid):
    """(cells, face_no) of the cell faces on boundary id `bid`: the faces
    whose (k+1)^(dim-1) nodes all carry the id (node_boundary bit), numbered
    as deal.II numbers the faces of a hex / quad, face_no = 2 * axis + side
    (what a caller collects from cell->face(f)->boundary_id())."""
    n, k, dim = mesh.degree + 1, mesh.degree, mesh.dim
    on = ((np.asarray(mesh.node_boundary) >> bid) & 1).astype(bool)
    cn = np.asarray(mesh.cell_nodes, dtype=np.int64)
    p = np.arange(n ** dim)
    ia = [p % n, (p // n) % n, p // (n * n)]
    cells, faces = [], []
    for a in range(dim):
        for side in range(2):
            sel = ia[a] == side * k
            hit = np.nonzero(on[cn[:, sel]].all(axis=1))[0]
            cells.append(hit)
            faces.append(np.full(len(hit), 2 * a + side))
    cells = np.concatenate(cells).astype(np.int64)
    faces = np.concatenate(faces).astype(np.int32)
    order = np.lexsort((faces, cells))
    return cells[order], faces[order]


# --------------------------------------------------------------------- decks
# the five input decks of the reference (input/*.json), shipped as package data
DECK_DIR = os.path.normpath(os.path.join(_HERE, "..", "data", "decks"))


@dataclass
class Deck:
    """Parameters of one input deck that reach the hot path (defaults as
    Parameters main.cc:66-118 and SimulationCylinder simulation.cc:198-222)."""
    name: str
    dim: int = 2
    fe_degree: int = 1
    n_refinements: int = 0
    simulation: str = "cylinder"
    time_integration: str = "bdf"
    bdf_order: int = 2
    theta: float = 1.0
    c1: float = 1.0
    c2: float = 1.0
    nu: float = 0.001
    consider_time_derivative: bool = True
    cell_wise_stabilization: bool = False
    nonlinear_solver: str = "Newton"
    no_slip_cylinder: bool = True
    no_slip_wall: bool = True
    cylinder_shift: float = 0.005
    u_max: float = 1.0
    t_init: float = 0.0
    outflow_bc: object = None  # override of the deck's outflow switches ("" = none)
    raw: dict = field(default_factory=dict)

    @property
    def increment_form(self):
        # main.cc:331
        return self.nonlinear_solver == "Newton"

    @property
    def outflow(self):
        """The outflow boundary (id 1) treatment of SimulationCylinder
        (simulation.cc:270-278, 394-403): "cut" (weak, all_outflow_bcs_cut),
        "nitsche" (weak, all_outflow_bcs_nitsche with the inflow function as
        target), "strong" (inhomogeneous Dirichlet with the inflow function)
        or None (homogeneous Neumann: the pressure is constrained).  A
        dataclass-level override (deck.outflow_bc = ...) wins."""
        if self.outflow_bc is not None:
            return self.outflow_bc or None
        r = self.raw
        if r.get("simulation use outflow bc weak cut", False):
            return "cut"
        if r.get("simulation use outflow bc weak nitsche", False):
            return "nitsche"
        if r.get("simulation use outflow bc strong", False):
            return "strong"
        return None

    def outflow_faces(self, mesh):
        """(cells, face_no) of the weak outflow faces (boundary id 1), or None."""
        if self.simulation != "cylinder" or self.outflow not in ("cut", "nitsche"):
            return None
        return boundary_faces(mesh, 1)

    def inflow_velocity(self, points, t=0.0, height=0.41):
        """InflowBoundaryValues::Channel (simulation.cc:25-76, built at
        simulation.cc:384-392) at points [..., dim]: velocity [..., dim]
        (component 0 only).  Also the Nitsche outflow target
        (simulation.cc:398) and the strong outflow's Dirichlet values."""
        x = np.asarray(points, dtype=np.float64)
        factor = np.ones(x.shape[:-1])
        if self.t_init != 0:  # ramp up
            factor *= min(t / self.t_init, 1.0)
        if self.no_slip_wall:  # parabolic profile
            H = height
            shift = -H / 2.0 + self.cylinder_shift
            y = x[..., 1] - shift
            factor *= 4 * y * (H - y) / H / H
            if x.shape[-1] == 3:
                z = x[..., 2] + H / 2.0
                factor *= 4 * z * (H - z) / H / H
        v = np.zeros(x.shape)
        v[..., 0] = self.u_max * factor
        return v

    @property
    def coarse_solver(self):
        # "gmg coarse grid solver" (multigrid.cc:164-166; default "AMG",
        # multigrid.h:35)
        return self.raw.get("gmg coarse grid solver", "AMG")

    def amg_parameters(self):
        """glsAMGParams keywords of the deck's coarse AMG (multigrid.cc:
        372-433): "gmg coarse grid amg use default parameters" true ->
        PreconditionAMG::AdditionalData() (one constant mode, threshold 1e-4,
        elliptic, Chebyshev smoother, Amesos-KLU coarse); false -> the
        multigrid.h:44-53 values (constant modes per component, threshold
        1e-14, non-elliptic, 2 sweeps; the ILU smoother / coarse solver are
        substituted by Chebyshev / a dense direct solve)."""
        if self.raw.get("gmg coarse grid amg use default parameters", True):
            return dict(block_size=1, threshold=1e-4, smoother_sweeps=2, coarse_max_size=2000,
                        elliptic=True, max_levels=10)
        return dict(block_size=self.dim + 1, threshold=1e-14, smoother_sweeps=2,
                    coarse_max_size=2000, elliptic=False, max_levels=10)

    @property
    def use_fe_q_iso_q1(self):
        # "gmg coarse grid use fe q iso q1" (main.cc:136, 436-446)
        return bool(self.raw.get("gmg coarse grid use fe q iso q1", False))

    def boundary_descriptor(self):
        """(vel_ids, p_ids, slip_ids) of constraints_homogeneous
        (simulation.cc:378-431 + main.cc:259-291)."""
        if self.simulation == "sphere":
            # simulation.cc:876-893: sphere (0) no-slip, inflow (1) Dirichlet,
            # walls (2) slip, outflow (3) pressure
            return [0, 1], [3], [2]
        if self.simulation != "cylinder":
            raise NotImplementedError(f"simulation {self.simulation!r} (SURVEY §8f next-4)")
        vel = [0]  # inflow: inhomogeneous DBC, zero in constraints_homogeneous
        slip = []
        walls = list(range(3, 3 + 2 * self.dim))
        (vel if self.no_slip_wall else slip).extend(walls)
        (vel if self.no_slip_cylinder else slip).append(2)
        p = []
        if self.outflow is None:
            p = [1]  # outflow: homogeneous "NBC" constrains the pressure
        elif self.outflow == "strong":
            vel.append(1)  # inhomogeneous DBC with the inflow function
        return vel, p, slip

    def constraint_values(self, mesh, t=0.0):
        """The inhomogeneity of constraints_inhomogeneous at time t
        (main.cc:879-891, 926-942) as a dof vector: the inflow function
        InflowBoundaryValues::Channel (simulation.cc:25-76, built at
        simulation.cc:384-392) interpolated at the support points of the
        velocity components on boundary id 0.  interpolate_boundary_values
        into an AffineConstraints skips dofs already constrained by
        constraints_copy (walls, cylinder, slip, outflow pressure), which
        keep the value 0.  Nonzero only on constrained components."""
        if self.simulation not in ("cylinder", "sphere"):
            raise NotImplementedError(f"simulation {self.simulation!r} (SURVEY §8f next-4)")
        vel, p, slip = self.boundary_descriptor()
        inflow_id = 1 if self.simulation == "sphere" else 0
        full = mesh.constraint_mask(vel, p, slip)
        inhom = {inflow_id} | ({1} if self.simulation == "cylinder" and self.outflow == "strong"
                               else set())
        copy = mesh.constraint_mask([i for i in vel if i not in inhom], p, slip)
        inflow = ((mesh.node_boundary >> inflow_id) & 1) != 0
        if self.simulation == "sphere":  # Channel(0.0, 1.0): uniform, u_max 1
            g = np.zeros(mesh.n_dofs)
            sel = inflow & ((full & 1) != 0) & ((copy & 1) == 0)
            g[np.nonzero(sel)[0] * (mesh.dim + 1)] = 1.0
            return g
        v = self.inflow_velocity(mesh.coords, t, mesh.params["height"])
        g = np.zeros(mesh.n_dofs)
        nc = mesh.dim + 1
        # component 0 carries u_max * factor, the other velocity components 0;
        # a strong outflow (id 1) takes the same function (simulation.cc:399-401)
        sel = inflow & ((full & 1) != 0) & ((copy & 1) == 0)
        if self.outflow == "strong":
            sel |= (((mesh.node_boundary >> 1) & 1) != 0) & ((full & 1) != 0) & ((copy & 1) == 0)
        g[np.nonzero(sel)[0] * nc] = v[sel, 0]
        return g

    def time_integrator(self, dt=2.5e-4, n_steps=None):
        """(theta, weights[0..order], order, current_dt) of the deck's
        TimeIntegratorData after `n_steps` constant-dt updates (default: order,
        i.e. full order reached) — time_integration.cc:10-178."""
        if self.time_integration == "none":
            return 1.0, [0.0], 0, 1.0
        if self.time_integration == "theta":
            return self.theta, [1.0 / dt, -1.0 / dt], 1, dt
        order = self.bdf_order
        n_steps = order if n_steps is None else n_steps
        dts = [dt if i < n_steps else 0.0 for i in range(order)]
        w = [0.0] * (order + 1)
        eff = sum(1 for x in dts if x > 0)
        d = dts
        if eff == 3:
            w[1] = -(d[0] + d[1]) * (d[0] + d[1] + d[2]) / (d[0] * d[1] * (d[1] + d[2]))
            w[2] = d[0] * (d[0] + d[1] + d[2]) / (d[1] * d[2] * (d[0] + d[1]))
            w[3] = -d[0] * (d[0] + d[1]) / (d[2] * (d[1] + d[2]) * (d[0] + d[1] + d[2]))
            w[0] = -(w[1] + w[2] + w[3])
        elif eff == 2:
            w[0] = (2 * d[0] + d[1]) / (d[0] * (d[0] + d[1]))
            w[1] = -(d[0] + d[1]) / (d[0] * d[1])
            w[2] = d[0] / (d[1] * (d[0] + d[1]))
        elif eff == 1:
            w[0], w[1] = 1.0 / d[0], -1.0 / d[0]
        return 1.0, w, order, d[0]

    def operator_parameters(self, dt=2.5e-4):
        """Keyword arguments for NavierStokesOperator.set_parameters / Oracle."""
        theta, w, order, cdt = self.time_integrator(dt)
        return dict(nu=self.nu, c1=self.c1, c2=self.c2, theta=theta, w0=w[0], dt=cdt,
                    order=order, increment_form=self.increment_form,
                    consider_time_derivative=self.consider_time_derivative,
                    cell_wise_stabilization=self.cell_wise_stabilization), w

    def mesh(self, n_ref=None):
        n_ref = self.n_refinements if n_ref is None else n_ref
        if self.simulation == "sphere":
            return sphere(self.fe_degree, n_ref, self.raw.get("mesh file"))
        return cylinder(self.dim, self.fe_degree, n_ref, shift=self.cylinder_shift)


def read_deck(path):
    with open(path) as f:
        raw = json.load(f)
    d = Deck(name=os.path.basename(path), raw=raw)
    d.dim = int(raw.get("dim", 2))
    d.fe_degree = int(raw.get("fe degree", 1))
    d.n_refinements = int(raw.get("n global refinements", 0))
    d.simulation = raw.get("simulation name", "channel")
    d.time_integration = raw.get("time intration", "theta")
    d.bdf_order = int(raw.get("bdf order", 1))
    d.theta = float(raw.get("theta", 0.5))
    d.c1 = float(raw.get("c1", 4.0))
    d.c2 = float(raw.get("c2", 2.0))
    d.nu = float(raw.get("nu", 0.1))
    d.consider_time_derivative = bool(raw.get("consider time derivative", False))
    d.cell_wise_stabilization = bool(raw.get("cell wise stabilization", True))
    d.nonlinear_solver = raw.get("nonlinear solver", "linearized")
    d.no_slip_cylinder = bool(raw.get("simulation no slip cylinder", True))
    d.no_slip_wall = bool(raw.get("simulation no slip wall", True))
    d.cylinder_shift = float(raw.get("simulation geometry cylinder shift", 0.005))
    d.u_max = float(raw.get("simulation u max", 1.0))
    d.t_init = float(raw.get("simulation t init", 0.0))
    return d


# ------------------------------------------------------------ arbitrary order
def _rotations(dim):
    """Proper rotations of the reference cell: (axis permutation, flips)."""
    out = []
    for perm in itertools.permutations(range(dim)):
        sign = np.linalg.det(np.eye(dim)[list(perm)])
        for flips in itertools.product((1, -1), repeat=dim):
            if sign * np.prod(flips) > 0:
                out.append((perm, flips))
    return out


class ShuffledMesh:
    """A generated mesh in an arbitrary cell order, the way a deal.II
    DoFHandler / MatrixFree hands it over (operator_ns.cc:806-830 loops over
    MatrixFree's cell batches, whatever their order): cells shuffled, nodes
    renumbered by first touch in the new cell order (DoFHandler's
    enumeration), optionally every cell re-oriented by a random proper
    rotation of its local lexicographic numbering.  Duck-types Mesh for
    NavierStokesOperator and the multigrid; brick() asks the library to
    discover the bricks (glsOpDesc::brick = {-1,-1,-1})."""

    def __init__(self, mesh, seed=0, rotate=False):
        rng = np.random.default_rng(seed)
        self.base = mesh
        self.dim, self.degree = mesh.dim, mesh.degree
        self.n_cells, self.n_nodes = mesh.n_cells, mesh.n_nodes
        n = self.degree + 1
        self.cell_order = rng.permutation(mesh.n_cells)  # new cell -> old cell
        cn = np.asarray(mesh.cell_nodes, dtype=np.int64)[self.cell_order]
        if rotate:
            rots = _rotations(self.dim)
            pick = rng.integers(0, len(rots), mesh.n_cells)
            shp = (n,) * self.dim
            for r, (perm, flips) in enumerate(rots):
                sel = pick == r
                if not sel.any():
                    continue
                # local arrays indexed [z][y][x] (x fastest): axis a of the
                # cell is array axis dim-1-a
                a = cn[sel].reshape((-1,) + shp)
                axes = [0] + [1 + (self.dim - 1 - perm[self.dim - 1 - q]) for q in range(self.dim)]
                a = a.transpose(axes)
                for q in range(self.dim):
                    if flips[q] < 0:
                        a = np.flip(a, axis=1 + (self.dim - 1 - q))
                cn[sel] = a.reshape(a.shape[0], -1)
        # first-touch node numbering in the new cell order
        flat = cn.ravel()
        _, first = np.unique(flat, return_index=True)
        order_old = flat[np.sort(first)]               # old nodes in first-touch order
        self.node_old = order_old                      # new node -> old node
        new_of_old = np.empty(mesh.n_nodes, dtype=np.int64)
        new_of_old[order_old] = np.arange(len(order_old))
        self.new_of_old = new_of_old
        self.cell_nodes = new_of_old[cn].astype(np.uint32)
        self.coords = np.asarray(mesh.coords)[order_old]
        self.node_boundary = np.asarray(mesh.node_boundary)[order_old]
        self._cached = None

    @property
    def n_dofs(self):
        return self.n_nodes * (self.dim + 1)

    def brick(self):
        return (-1, -1, -1)

    def cell_measure(self):
        meas, hmin = self.base.cell_measure()
        return meas[self.cell_order], hmin[self.cell_order]

    def constraint_mask(self, *a, **k):
        return np.asarray(self.base.constraint_mask(*a, **k))[self.node_old]

    def child_lattice(self, fine):
        """Child lattices of this (coarse) level's cells into `fine` (both
        shuffled views of consecutive generator levels)."""
        ch = np.asarray(self.base.child_lattice(fine.base), dtype=np.int64)
        return fine.new_of_old[ch[self.cell_order]].astype(np.uint32)


# ------------------------------------------------------------ FE_Q_iso_Q1
def _gll_nodes(k):
    """Support points of FE_Q(k) / MappingQ(k) on [0, 1] (QGaussLobatto(k+1))."""
    if k == 1:
        return np.array([0.0, 1.0])
    if k == 2:
        return np.array([0.0, 0.5, 1.0])
    if k == 3:
        r = np.sqrt(5.0) / 10.0
        return np.array([0.0, 0.5 - r, 0.5 + r, 1.0])
    raise ValueError("degree > 3 not supported")


def _lagrange(nodes, i, x):
    v = np.ones_like(np.asarray(x, dtype=np.float64))
    for j, xj in enumerate(nodes):
        if j != i:
            v = v * (x - xj) / (nodes[i] - xj)
    return v


class IsoQ1Mesh:
    """The multigrid's coarsest level with FE_Q_iso_Q1 (main.cc:436-446,
    "gmg coarse grid use fe q iso q1"): the same support points as FE_Q(k)
    on the coarse cells, the basis piecewise linear on the k^dim sub-cells of
    every cell, quadrature QIterated(QGauss(2), k) — which is the Q1 operator
    on the sub-cells with QGauss(2), on the unchanged node numbering.  So the
    level is a degree-1 NavierStokesOperator over the sub-cells (k^dim per
    coarse cell, lexicographic, a k x k (x k) brick each); the penalty
    parameters keep the coarse cell's (operator_ns.cc:399-407: measure /
    fe_degree with fe_degree = k — here the sub-cell measure |K| / k^dim at
    degree 1 — and the cell's minimum vertex distance).  The transfer to the
    next level is the Q1 one: every sub-cell is one child of the next level,
    whose Q_k nodes sit at the sub-cell's 3^dim refined lattice points
    (child_lattice), and the linear embedding is the iso-Q1 prolongation.
    Geometry: the parent cell's MappingQ(k) at the iterated quadrature
    points (mapping_points: per sub-cell the parent map at its Q_k lattice,
    passed to the operator as glsOpDesc.mapping_points), as the reference
    maps every level with MappingQ(mapping_degree) (main.cc:413-414)."""

    def __init__(self, mesh):
        k, dim = mesh.degree, mesh.dim
        if k < 2:
            raise ValueError("FE_Q_iso_Q1 needs a coarse element of degree >= 2")
        self.base, self.k = mesh, k
        self.dim, self.degree = dim, 1
        self.n_nodes = mesh.n_nodes
        self.coords = mesh.coords
        n = k + 1
        cn = np.asarray(mesh.cell_nodes, dtype=np.int64).reshape((-1,) + (n,) * dim)  # [c][z][y][x]
        subs = []
        rng = range(k)
        if dim == 3:
            for a in rng:            # sub-cell z
                for b in rng:        # y
                    for c in rng:    # x
                        corners = [cn[:, a + l, b + j, c + i] for l in (0, 1) for j in (0, 1)
                                   for i in (0, 1)]
                        subs.append(np.stack(corners, axis=1))
        else:
            for b in rng:
                for c in rng:
                    corners = [cn[:, b + j, c + i] for j in (0, 1) for i in (0, 1)]
                    subs.append(np.stack(corners, axis=1))
        # [coarse cell][sub-cell lexicographic][2^dim]
        self.cell_nodes = np.ascontiguousarray(np.stack(subs, axis=1).reshape(-1, 2 ** dim),
                                               dtype=np.uint32)
        self.n_cells = self.cell_nodes.shape[0]
        self.n_sub = k ** dim

    @property
    def n_dofs(self):
        return self.n_nodes * (self.dim + 1)

    def brick(self):
        return (self.k, self.k, self.k if self.dim == 3 else 1)

    def mapping_points(self):
        """The level's MappingQ(k) (main.cc:413-414: one mapping of the
        level's degree for every level, the FE_Q_iso_Q1 coarse level too)
        restricted to each sub-cell: the parent's Q_k map evaluated at the
        sub-cell's (k+1)^dim GLL lattice points.  A Q_k map restricted to a
        sub-box is again a Q_k map of the sub-cell's own coordinates, so these
        points reproduce the parent mapping at the iterated quadrature points
        exactly (curved cells included).  Returns (k, [n_cells][(k+1)^dim][dim])."""
        k, dim = self.k, self.dim
        n = k + 1
        g = _gll_nodes(k)                      # parent and sub-cell lattices
        # E[c][j][i]: parent basis i at sub-cell c's lattice point j (1D)
        E = np.zeros((k, n, n))
        for c in range(k):
            xi = g[c] + (g[c + 1] - g[c]) * g
            for i in range(n):
                E[c, :, i] = _lagrange(g, i, xi)
        X = np.asarray(self.coords, dtype=np.float64)[
            np.asarray(self.base.cell_nodes, dtype=np.int64)].reshape((-1,) + (n,) * dim + (dim,))
        out = []
        if dim == 3:
            for a in range(k):
                for b in range(k):
                    for c in range(k):
                        out.append(np.einsum("pz,qy,rx,nzyxd->npqrd", E[a], E[b], E[c], X)
                                   .reshape(X.shape[0], -1, dim))
        else:
            for b in range(k):
                for c in range(k):
                    out.append(np.einsum("qy,rx,nyxd->nqrd", E[b], E[c], X)
                               .reshape(X.shape[0], -1, dim))
        pts = np.stack(out, axis=1).reshape(-1, n ** dim, dim)  # [coarse][sub] order
        return k, np.ascontiguousarray(pts)

    def cell_measure(self):
        meas, hmin = self.base.cell_measure()
        return (np.repeat(np.asarray(meas) / self.n_sub, self.n_sub),
                np.repeat(np.asarray(hmin), self.n_sub))

    def constraint_mask(self, *a, **kw):
        return self.base.constraint_mask(*a, **kw)

    def child_lattice(self, fine):
        """Per sub-cell, the 3^dim next-level nodes of its child (the
        sub-block of the coarse cell's (2k+1)^dim child lattice)."""
        k, dim = self.k, self.dim
        L = 2 * k + 1
        ch = np.asarray(self.base.child_lattice(fine), dtype=np.int64).reshape((-1,) + (L,) * dim)
        out = []
        if dim == 3:
            for a in range(k):
                for b in range(k):
                    for c in range(k):
                        out.append(ch[:, 2 * a:2 * a + 3, 2 * b:2 * b + 3, 2 * c:2 * c + 3]
                                   .reshape(ch.shape[0], -1))
        else:
            for b in range(k):
                for c in range(k):
                    out.append(ch[:, 2 * b:2 * b + 3, 2 * c:2 * c + 3].reshape(ch.shape[0], -1))
        return np.ascontiguousarray(np.stack(out, axis=1).reshape(-1, 3 ** dim), dtype=np.uint32)
