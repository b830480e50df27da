"""Multi-GPU driver of the GLS operator: one process per GPU, cells partitioned
into contiguous brick ranges (x-slabs of the cylinder mesh), ghost DoFs
exchanged point-to-point over torch.distributed (RCCL on MI355X, gloo on CPU).

Reference behaviour restated (deal.II distributed vectors inside
MatrixFree::cell_loop, operator_ns.cc:702-721 / operator_base.cc:684-732):

  vmult(dst, src):
    src.update_ghost_values()        owner -> ghost copies   (import)
    dst = 0; cell loop over the locally owned cells, ghost rows collect
          partial sums
    dst.compress(VectorOperation::add)   ghost partials -> owner, added;
                                         ghost entries zeroed  (export-add)
    dst[c] = src[c] for constrained owned dofs   (identity rows, :719-721)

Ownership: a node belongs to the lowest rank whose cells touch it (deal.II's
"lowest subdomain id owns the interface" rule); local layout [owned | ghost],
owned in mesh order, ghosts grouped by owner so every import lands in one
contiguous block.  The partition is computed identically on every rank from
the replicated mesh (no exchange of the plan).

Two transports:
  * native (the product path on GPUs): libglsamd.so's gls_dist_* — pack
    kernel, RCCL send/recv of the ghost blocks on a communication stream
    while the interior bricks (those reading no ghost node) run, boundary
    bricks after the import event, export-add over RCCL, one unpack-add
    kernel.  In-process groups (LocalGroup, one device) run the same phases
    with device copies in place of RCCL.
  * torch.distributed point-to-point (batch_isend_irecv) with the per-rank
    phases below (pack / unpack / local apply / fix): the CPU/gloo tests (the
    tests inject a CPU oracle engine, tests/dist_engines.py) and the
    cross-check of the native path.
"""
from __future__ import annotations

import numpy as np


# ------------------------------------------------------------------ partition
class Partition:
    """Host-side plan of one rank: local cells/nodes and exchange lists."""

    def __init__(self, rank, world, cell_range, local_nodes, n_owned, owner):
        self.rank, self.world = rank, world
        self.cell_begin, self.cell_end = cell_range
        self.local_nodes = local_nodes        # global ids, local order
        self.n_owned = n_owned
        self.n_nodes = len(local_nodes)
        self.node_owner = owner[local_nodes]  # owner of each local node
        # filled by build_partitions
        self.recv_nodes = {}  # q -> my ghost local indices owned by q (gid order)
        self.send_nodes = {}  # q -> my owned local indices that are ghosts on q

    @property
    def n_cells(self):
        return self.cell_end - self.cell_begin


def _brick_cells(mesh):
    b = mesh.brick()
    n = 1
    for x in b[:mesh.dim]:
        n *= max(1, x)
    return n


def coarse_bounds(n_coarse_cells, world):
    """Contiguous ranges of coarse (level 0) cells per rank: every level of a
    hierarchy is partitioned by the same coarse cells (the children of a
    rank's coarse cells are its fine cells), as p4est's partition of the
    coarse forest keeps the levels aligned (main.cc:398-400)."""
    if world > n_coarse_cells:
        raise ValueError(f"{world} ranks for {n_coarse_cells} coarse cells")
    return [r * n_coarse_cells // world for r in range(world + 1)]


def build_partitions(mesh, world, bounds=None):
    """Split the cell list into `world` contiguous brick ranges (or the given
    cell `bounds`) and derive the ownership / ghost / exchange plan for every
    rank."""
    if bounds is None:
        nbc = _brick_cells(mesh)
        if mesh.n_cells % nbc:
            raise ValueError("cell count is not a multiple of the brick size")
        nb = mesh.n_cells // nbc
        if world > nb:
            raise ValueError(f"{world} ranks for {nb} bricks")
        bounds = [(r * nb // world) * nbc for r in range(world + 1)]
    bounds = [int(b) for b in bounds]
    touched = [np.unique(mesh.cell_nodes[bounds[r]:bounds[r + 1]].ravel())
               for r in range(world)]
    owner = np.full(mesh.n_nodes, world, dtype=np.int64)
    for r in range(world - 1, -1, -1):
        owner[touched[r]] = r
    parts = []
    for r in range(world):
        t = touched[r]
        own = t[owner[t] == r]
        gh = t[owner[t] != r]
        gh = gh[np.lexsort((gh, owner[gh]))]  # by (owner, gid)
        local = np.concatenate([own, gh]).astype(np.int64)
        parts.append(Partition(r, world, (bounds[r], bounds[r + 1]), local, len(own), owner))
    g2l = []
    for p in parts:
        m = np.full(mesh.n_nodes, -1, dtype=np.int64)
        m[p.local_nodes] = np.arange(p.n_nodes)
        g2l.append(m)
    for p in parts:
        ghosts = p.local_nodes[p.n_owned:]
        gown = p.node_owner[p.n_owned:]
        for q in np.unique(gown):
            q = int(q)
            gids = ghosts[gown == q]  # sorted by gid (lexsort above)
            p.recv_nodes[q] = g2l[p.rank][gids]
            parts[q].send_nodes[p.rank] = g2l[q][gids]
    return parts


def _dofs(nodes, nc):
    nodes = np.asarray(nodes, dtype=np.int64)
    return (nodes[:, None] * nc + np.arange(nc)[None, :]).ravel()


def _cu_count():
    try:
        import torch
        return torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    except Exception:
        return 256


def _local_brick(b, n_cells):
    """A rank whose layer bricks (bx x by x 1) number fewer than the GPU's
    CUs runs half-height bricks (bx x by/2 x 1, consecutive in the cell
    order): more, shorter work units for a GPU the strong-scaled slab no
    longer fills (Re3900 r2 at 8 ranks, 3,200 cells: 14.1 -> 12.5 us per
    local vmult, scripts/dist_brick_sweep.py)."""
    b = tuple(int(x) for x in b)
    cells = b[0] * max(b[1], 1) * max(b[2], 1)
    if (len(b) == 3 and b[2] == 1 and b[1] % 2 == 0 and b[0] > 0 and cells > 0
            and n_cells % cells == 0 and n_cells // cells < _cu_count()):
        return (b[0], b[1] // 2, 1)
    return b


class LocalMesh:
    """The rank-local view of a mesh with the attributes NavierStokesOperator /
    OracleMesh read (duck-typed glsmesh.Mesh)."""

    def __init__(self, mesh, part: Partition):
        self.dim, self.degree = mesh.dim, mesh.degree
        self.n_nodes = part.n_nodes
        self.n_cells = part.n_cells
        g2l = np.full(mesh.n_nodes, -1, dtype=np.int64)
        g2l[part.local_nodes] = np.arange(part.n_nodes)
        cn = mesh.cell_nodes[part.cell_begin:part.cell_end]
        self.cell_nodes = g2l[cn].astype(np.uint32)
        self.coords = np.ascontiguousarray(mesh.coords[part.local_nodes])
        meas, hmin = mesh.cell_measure()
        self._meas = np.ascontiguousarray(meas[part.cell_begin:part.cell_end])
        self._hmin = np.ascontiguousarray(hmin[part.cell_begin:part.cell_end])
        self._brick = _local_brick(mesh.brick(), self.n_cells)
        mp = getattr(mesh, "mapping_points", None)
        self._mapping = None
        if callable(mp):
            m, pts = mp()
            self._mapping = (m, np.ascontiguousarray(pts[part.cell_begin:part.cell_end]))

    def mapping_points(self):
        return self._mapping

    @property
    def n_dofs(self):
        return self.n_nodes * (self.dim + 1)

    def cell_measure(self):
        return self._meas, self._hmin

    def brick(self):
        return self._brick


# ------------------------------------------------------------------ engines
def recv_blocks(part: Partition):
    """Per owner q: (first local ghost node, count) — ghosts of one owner are
    one contiguous block of the local layout."""
    out = {}
    for q, idx in part.recv_nodes.items():
        idx = np.asarray(idx, dtype=np.int64)
        if len(idx) and not np.array_equal(idx, np.arange(idx[0], idx[0] + len(idx))):
            raise ValueError("ghosts of one owner are not contiguous")
        out[q] = (int(idx[0]) if len(idx) else part.n_owned, len(idx))
    return out


class GpuEngine:
    """Local operator = libglsamd.so (the product path)."""

    def __init__(self, lmesh, cmask, n_owned, precision):
        import glsamd
        self.op = glsamd.NavierStokesOperator(lmesh, cmask, precision, n_owned_nodes=n_owned,
                                              brick=lmesh.brick())
        self.dtype = self.op.dtype
        self.device = "cuda"

    def set_parameters(self, **params):
        self.op.set_parameters(**params)

    def set_linearization_point(self, v):
        self.op.set_linearization_point(v)

    def set_previous_solution(self, hist, w):
        self.op.set_previous_solution(hist, w)

    def local_vmult(self, dst, src):
        self.op.vmult(dst, src)

    def identity_rows(self, dst, src):
        self.op.apply_identity_rows(dst, src)

    def diagonal_raw(self, d):
        self.op.compute_diagonal(d)

    def invert_diagonal(self, d):
        self.op.invert_diagonal(d)

    def partitioned(self, part, nccl_id=None, group=None):
        import glsamd
        peers = sorted(set(part.recv_nodes) | set(part.send_nodes))
        send = {q: part.send_nodes.get(q, np.zeros(0, np.int64)) for q in peers}
        rb = recv_blocks(part)
        recv = {q: rb.get(q, (part.n_owned, 0)) for q in peers}
        return glsamd.PartitionedOperator(self.op, part.rank, part.world, peers, send, recv,
                                          nccl_id=nccl_id, group=group)


# ------------------------------------------------------------------ rank state
class RankOperator:
    """One rank's share of the distributed operator (phases of vmult)."""

    def __init__(self, mesh, cmask, part: Partition, precision="f64", engine="gpu"):
        import torch
        self.part = part
        self.nc = mesh.dim + 1
        self.lmesh = LocalMesh(mesh, part)
        lcmask = np.ascontiguousarray(cmask[part.local_nodes], dtype=np.uint8)
        # engine: "gpu" (the product path) or a local-operator factory with
        # GpuEngine's interface (the CPU tests inject the oracle,
        # tests/dist_engines.py)
        cls = GpuEngine if engine == "gpu" else engine
        self.eng = cls(self.lmesh, lcmask, part.n_owned, precision)
        self.dtype, self.device = self.eng.dtype, self.eng.device
        self.n_dofs = part.n_nodes * self.nc
        self.n_owned_dofs = part.n_owned * self.nc
        cmo = np.asarray(lcmask[:part.n_owned], dtype=np.int64)
        self.con_owned = torch.from_numpy(
            (((cmo[:, None] >> np.arange(self.nc)[None, :]) & 1) != 0).ravel()).to(self.device)
        self.global_dofs = torch.from_numpy(_dofs(part.local_nodes, self.nc)).to(self.device)
        dev = lambda a: torch.from_numpy(_dofs(a, self.nc)).to(self.device)  # noqa: E731
        self.recv_idx = {q: dev(v) for q, v in part.recv_nodes.items()}
        self.send_idx = {q: dev(v) for q, v in part.send_nodes.items()}
        self.peers = sorted(set(self.recv_idx) | set(self.send_idx))
        z = lambda n: torch.empty(n, dtype=self.dtype, device=self.device)  # noqa: E731
        self.recv_buf = {q: z(len(v)) for q, v in self.recv_idx.items()}
        self.send_buf = {q: z(len(v)) for q, v in self.send_idx.items()}
        # export-add reuses the import lists in the opposite direction
        self.xrecv_buf = {q: z(len(v)) for q, v in self.send_idx.items()}
        self.xsend_buf = {q: z(len(v)) for q, v in self.recv_idx.items()}

    @property
    def op(self):
        return getattr(self.eng, "op", None)

    def new_vector(self):
        import torch
        return torch.zeros(self.n_dofs, dtype=self.dtype, device=self.device)

    def local_from_global(self, g):
        """Local [owned | ghost] vector from a replicated global vector."""
        import torch
        g = torch.as_tensor(np.asarray(g) if not torch.is_tensor(g) else g)
        return g.to(self.device, self.dtype)[self.global_dofs].contiguous()

    # import: owned -> ghosts of the peers
    def pack_import(self, v):
        for q, idx in self.send_idx.items():
            torch_index_select(v, idx, self.send_buf[q])
        return self.send_buf, self.recv_buf

    def unpack_import(self, v):
        for q, idx in self.recv_idx.items():
            v.index_copy_(0, idx, self.recv_buf[q])

    # export-add: ghost partials -> owners
    def pack_export(self, v):
        for q, idx in self.recv_idx.items():
            torch_index_select(v, idx, self.xsend_buf[q])
        return self.xsend_buf, self.xrecv_buf

    def unpack_export(self, v):
        for q, idx in self.send_idx.items():
            v.index_add_(0, idx, self.xrecv_buf[q])
        v[self.n_owned_dofs:].zero_()


def torch_index_select(v, idx, out):
    import torch
    torch.index_select(v, 0, idx, out=out)


# ------------------------------------------------------------------ drivers
class DistributedOperator:
    """NavierStokesOperator over a torch.distributed process group: the
    OperatorBase calls the reference's NonlinearSolver / GMRES make on a
    distributed operator (set_linearization_point, set_previous_solution,
    vmult), on rank-local [owned | ghost] vectors."""

    def __init__(self, mesh, cmask, precision, dist, rank, world, engine="gpu", native=None,
                 bounds=None):
        self.dist, self.rank, self.world = dist, rank, world
        self.parts = build_partitions(mesh, world, bounds)
        self.r = RankOperator(mesh, cmask, self.parts[rank], precision, engine)
        self.n_local_cells = self.r.part.n_cells
        self.n_global_dofs = mesh.n_dofs
        self.native = None
        if native is None:
            native = engine == "gpu"
        if native:
            self.native = self.r.eng.partitioned(self.r.part, nccl_id=self._shared_id())

    def _shared_id(self):
        """RCCL unique id from rank 0, broadcast over the torch process group."""
        import torch
        import glsamd
        dev = "cuda" if self.dist.get_backend() == "nccl" else "cpu"
        t = torch.zeros(128, dtype=torch.uint8, device=dev)
        if self.rank == 0:
            t.copy_(torch.frombuffer(bytearray(glsamd.dist_unique_id()), dtype=torch.uint8))
        self.dist.broadcast(t, 0)
        return bytes(t.cpu().numpy().tobytes())

    @property
    def op(self):
        return self.r.op

    def new_vector(self):
        return self.r.new_vector()

    def scatter_global(self, g):
        return self.r.local_from_global(g)

    def _exchange(self, sends, recvs):
        d = self.dist
        ops = [d.P2POp(d.irecv, buf, q) for q, buf in recvs.items()]
        ops += [d.P2POp(d.isend, buf, q) for q, buf in sends.items()]
        if ops:
            for w in d.batch_isend_irecv(ops):
                w.wait()

    def update_ghost_values(self, v):
        if self.native is not None:
            return self.native.update_ghost_values(v)
        sends, recvs = self.r.pack_import(v)
        self._exchange(sends, recvs)
        self.r.unpack_import(v)

    def compress_add(self, v):
        if self.native is not None:
            return self.native.compress_add(v)
        sends, recvs = self.r.pack_export(v)
        self._exchange(sends, recvs)
        self.r.unpack_export(v)

    def setup(self, params, u_star, hist=None, weights=None):
        """set_parameters + set_linearization_point (+ set_previous_solution)
        from replicated global vectors; ghost values are imported from their
        owners, as a distributed solution vector's update_ghost_values."""
        self.dist.barrier()
        eng = self.r.eng
        eng.set_parameters(**params)
        u = self._owned_then_import(u_star)
        eng.set_linearization_point(u)
        if hist is not None and params.get("order", 0) > 0:
            eng.set_previous_solution([self._owned_then_import(h) for h in hist], weights)

    def _owned_then_import(self, g):
        v = self.scatter_global(g)
        v[self.r.n_owned_dofs:].zero_()
        self.update_ghost_values(v)
        return v

    def vmult(self, dst, src):
        if self.native is not None:
            return self.native.vmult(dst, src)
        return self.vmult_p2p(dst, src)

    def vmult_p2p(self, dst, src):
        self.update_ghost_values(src)
        self.r.eng.local_vmult(dst, src)
        self.compress_add(dst)
        self.r.eng.identity_rows(dst, src)
        return dst

    def gather_global(self, v):
        """Replicated global (mesh-numbered) vector of the owned entries."""
        import torch
        g = torch.zeros(self.n_global_dofs, dtype=v.dtype, device=v.device)
        n = self.r.n_owned_dofs
        g.index_copy_(0, self.r.global_dofs[:n], v[:n])
        self.dist.all_reduce(g)
        return g


def run_threaded(world, fn):
    """fn(rank) on `world` host threads, each with its own torch stream as
    the current stream (the members of an in-process group driven the way
    RCCL ranks are: one rank call sequence per thread, libglsamd's
    production schedule with device copies as transport; ctypes releases
    the GIL inside the calls).  Returns the results in rank order; the first
    exception of any thread is re-raised."""
    import threading
    import torch
    torch.cuda.synchronize()
    dev = torch.cuda.current_device()
    out, err = [None] * world, [None] * world

    def body(r):
        try:
            torch.cuda.set_device(dev)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                out[r] = fn(r)
            st.synchronize()
        except BaseException as e:  # noqa: BLE001 (re-raised below)
            err[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in err:
        if e is not None:
            raise e
    torch.cuda.synchronize()
    return out


class LocalGroup:
    """All ranks of a partition in ONE process (one device): the same phases
    with direct buffer delivery instead of point-to-point messages.  Used to
    test the partitioned operator on a single GPU."""

    def __init__(self, mesh, cmask, world, precision="f64", engine="gpu", native=False):
        self.parts = build_partitions(mesh, world)
        self.ranks = [RankOperator(mesh, cmask, p, precision, engine) for p in self.parts]
        self.n_global_dofs = mesh.n_dofs
        self.native = None
        if native:
            self.native = []
            for r in self.ranks:
                g = self.native[0] if self.native else None
                self.native.append(r.eng.partitioned(r.part, group=g))

    def _deliver(self, packs):
        for r, (sends, _) in enumerate(packs):
            for q, buf in sends.items():
                packs[q][1][r].copy_(buf)

    def update_ghost_values(self, vs):
        self._deliver([r.pack_import(v) for r, v in zip(self.ranks, vs)])
        for r, v in zip(self.ranks, vs):
            r.unpack_import(v)

    def compress_add(self, vs):
        self._deliver([r.pack_export(v) for r, v in zip(self.ranks, vs)])
        for r, v in zip(self.ranks, vs):
            r.unpack_export(v)

    def setup(self, params, u_star, hist=None, weights=None):
        for r in self.ranks:
            r.eng.set_parameters(**params)
        us = self.scatter(u_star)
        for r, u in zip(self.ranks, us):
            r.eng.set_linearization_point(u)
        if hist is not None and params.get("order", 0) > 0:
            hs = [self.scatter(h) for h in hist]
            for i, r in enumerate(self.ranks):
                r.eng.set_previous_solution([h[i] for h in hs], weights)

    def scatter(self, g):
        vs = [r.local_from_global(g) for r in self.ranks]
        for r, v in zip(self.ranks, vs):
            v[r.n_owned_dofs:].zero_()
        self.update_ghost_values(vs)
        return vs

    def vmult_threaded(self, dsts, srcs, reps=1):
        """gls_dist_vmult per member from its own thread and stream (the
        production two-stream schedule of an RCCL rank), `reps` times"""
        def one(r):
            for _ in range(reps):
                self.native[r].vmult(dsts[r], srcs[r])
        run_threaded(len(self.ranks), one)
        return dsts

    def vmult(self, dsts, srcs):
        if self.native is not None:
            import glsamd
            return glsamd.PartitionedOperator.vmult_group(self.native, dsts, srcs)
        self.update_ghost_values(srcs)
        for r, d, s in zip(self.ranks, dsts, srcs):
            r.eng.local_vmult(d, s)
        self.compress_add(dsts)
        for r, d, s in zip(self.ranks, dsts, srcs):
            r.eng.identity_rows(d, s)
        return dsts

    def gather(self, vs):
        import torch
        g = torch.zeros(self.n_global_dofs, dtype=vs[0].dtype, device=vs[0].device)
        for r, v in zip(self.ranks, vs):
            n = r.n_owned_dofs
            g.index_copy_(0, r.global_dofs[:n], v[:n])
        return g


# ------------------------------------------------------------ multigrid
def global_first_owners(child):
    """NOT_OWNER flags (bit 31) of a global child lattice [coarse cell][nl]:
    the first coarse cell (global order) touching a fine node owns it — the
    owner-only transfers of csrc/mg.hip, and with ranks holding contiguous
    coarse-cell ranges the owner cell of every fine node lies on the rank that
    owns the node (the lowest rank touching it)."""
    flat = np.asarray(child, dtype=np.int64).ravel()
    _, first = np.unique(flat, return_index=True)
    owner = np.zeros(flat.shape, dtype=bool)
    owner[first] = True
    return owner.reshape(np.shape(child))


class DistributedMultigrid:
    """PreconditionerGMG (multigrid.h:61-141) over a partitioned level
    hierarchy, one process per GPU: every level is a DistributedOperator on
    the same coarse-cell partition (main.cc:398-400), the transfers run the
    owner-only lattice kernels on the rank-local cells with halo exchanges
    around them (MGTransferGlobalCoarsening's ghosted level vectors,
    main.cc:540-563):
        prolongate: update_ghost_values(coarse), local prolongate_add
                    (every owned fine node is written by its owner rank);
        restrict:   local restrict_add (owned fine nodes feed the coarse
                    nodes of their owner cell), compress(add) on the coarse
                    vector;
        interpolate_to_mg: update_ghost_values(fine), local injection.
    Smoother: PreconditionRelaxation (damped Jacobi, power-iteration omega
    with deal.II's start vector on the GLOBAL dof index and all-reduced
    dots, multigrid.cc:281-369); inverse diagonals from the rank-local
    assembled diagonals after compress(add).  Coarse solve: relaxation
    sweeps (the substitute for the direct solver) or
    identity.  engine: "gpu" (libglsamd.so kernels, RCCL exchange) or a test
    engine (tests/dist_engines.py) with the same interface."""

    def __init__(self, meshes, cmasks, precision, dist, rank, world, engine="gpu",
                 transfers=None, n_smooth=5, n_eig=20, smoothing_range=20.0,
                 coarse_n_iterations=10, compute_evs_n_levels=0, native=None,
                 coarse_solver=None):
        self.dist, self.rank, self.world = dist, rank, world
        # coarse_n_iterations < 0: the deck's direct coarse solver, redundant
        # on every rank (the coarse right-hand side all-gathered, SURVEY
        # §8e "the coarse level is gathered for the direct solve"):
        # coarse_solver (a factory taking the level-0 mesh, cmask, precision)
        # or RedundantCoarseLU
        self._coarse_direct = coarse_n_iterations < 0
        if self._coarse_direct:
            make = coarse_solver or RedundantCoarseLU
            self.coarse = make(meshes[0], cmasks[0], precision)
        self.n_smooth, self.n_eig, self.range = n_smooth, n_eig, smoothing_range
        self.coarse_iters, self.evs_levels = coarse_n_iterations, compute_evs_n_levels
        n0 = meshes[0].n_cells
        cb = coarse_bounds(n0, world)
        self.fine_bounds = [b * (meshes[-1].n_cells // n0) for b in cb]
        self._fine = (meshes[-1], cmasks[-1], engine, native)
        self._n_global_nodes = [m.n_nodes for m in meshes]
        self._coarse_mesh = (meshes[0], cmasks[0], precision)
        self._meshes = (list(meshes), list(cmasks), precision)
        self.levels = []
        for m, cm in zip(meshes, cmasks):
            if m.n_cells % n0:
                raise ValueError("level meshes must refine the coarse cells uniformly")
            ratio = m.n_cells // n0
            self.levels.append(DistributedOperator(m, cm, precision, dist, rank, world,
                                                   engine=engine, native=native,
                                                   bounds=[b * ratio for b in cb]))
        # rank-local child lattices (local fine node ids) with global-first
        # owner flags
        self.child = [None]
        for l in range(1, len(meshes)):
            G = np.asarray(meshes[l - 1].child_lattice(meshes[l]), dtype=np.int64)
            own = global_first_owners(G)
            pc = self.levels[l - 1].r.part
            pf = self.levels[l].r.part
            g2l = np.full(meshes[l].n_nodes, -1, dtype=np.int64)
            g2l[pf.local_nodes] = np.arange(pf.n_nodes)
            rows = G[pc.cell_begin:pc.cell_end]
            loc = g2l[rows]
            if (loc < 0).any():
                raise ValueError("a child lattice node is not local to the fine partition")
            ch = loc.astype(np.uint32)
            ch[~own[pc.cell_begin:pc.cell_end]] |= np.uint32(0x80000000)
            self.child.append(ch)
        if transfers is None:
            import glsamd
            transfers = glsamd.Multigrid([D.op for D in self.levels], self.child[1:],
                                         coarse_n_iterations=coarse_n_iterations,
                                         outer_precision=precision)
        elif callable(transfers) and not hasattr(transfers, "prolongate_add"):
            transfers = transfers(self)  # a factory (tests: numpy transfers)
        self.tr = transfers
        self.omega = [1.0] * len(self.levels)
        self.lam = [0.0] * len(self.levels)
        self.invdiag = [None] * len(self.levels)
        import torch
        self._global_dof = []
        for D in self.levels:
            gd = torch.from_numpy(_dofs(D.r.part.local_nodes[:D.r.part.n_owned], D.r.nc))
            self._global_dof.append(gd.to(D.r.device))

    def native(self, params, u_star, hist=None, weights=None, redundant_levels=0):
        """This rank's native partitioned multigrid over the same level
        operators (glsamd.PartitionedMultigrid, gls_dist_mg_*: the V-cycle
        with its halo exchanges, relaxation and coarse solve inside the
        library, one team call per rank) with its linearization point and
        setup done; the GMRES over it is glsamd.dist_gmres_solve([fine
        operator's native handle], [mg], ...).  Needs the native level
        operators (engine "gpu").  redundant_levels = k > 0: levels 0 .. k-1
        and a global copy of level k run single-domain on this rank (level
        agglomeration, glsDistMGDesc n_redundant_levels); the partitioned
        hierarchy starts at level k."""
        import glsamd
        k = int(redundant_levels)
        levels = self.levels[k:]
        hs = [D.native for D in levels]
        if any(h is None for h in hs):
            raise ValueError("native(): the level operators have no native handles")
        coarse, l2g, rops, rch = None, None, None, None
        keep = []
        if self._coarse_direct or k > 0:
            meshes, cmasks, prec = self._meshes
            coarse = glsamd.NavierStokesOperator(meshes[k], cmasks[k], prec)
            coarse.set_parameters(**params)
            l2g = levels[0].r.part.local_nodes
            keep.append(coarse)
            if k > 0:
                rops = [glsamd.NavierStokesOperator(meshes[l], cmasks[l], prec)
                        for l in range(k)]
                for o in rops:
                    o.set_parameters(**params)
                rch = [None] + [meshes[l - 1].child_lattice(meshes[l]) for l in range(1, k + 1)]
                keep += rops
        mg = glsamd.PartitionedMultigrid(
            hs, [None] + list(self.child[k + 1:]),
            [D.r.part.local_nodes[:D.r.part.n_owned] for D in levels],
            self._n_global_nodes[k:], smoothing_n_iterations=self.n_smooth,
            smoothing_eig_n_iterations=self.n_eig, smoothing_range=self.range,
            coarse_n_iterations=self.coarse_iters, compute_evs_n_levels=self.evs_levels,
            coarse_global=coarse, coarse_l2g=l2g, redundant_ops=rops, redundant_child=rch)
        mg._keep_ops = keep
        for D in levels:
            D.r.eng.set_parameters(**params)
        top = levels[-1].r
        u = [top.local_from_global(u_star)]
        h = None
        if hist is not None and params.get("order", 0) > 0:
            h = [[top.local_from_global(x) for x in hist]]
        glsamd.PartitionedMultigrid.set_linearization_point([mg], u, h, weights)
        glsamd.PartitionedMultigrid.setup([mg])
        return mg

    def fine_operator(self, precision="f64"):
        """The outer (system) operator on the finest level's partition: its
        rank-local vectors are the ones vmult() takes (the GMRES operand)."""
        m, cm, engine, native = self._fine
        return DistributedOperator(m, cm, precision, self.dist, self.rank, self.world,
                                   engine=engine, native=native, bounds=self.fine_bounds)

    # ---- vectors and reductions
    def new_vector(self, l):
        return self.levels[l].new_vector()

    def _owned(self, l, v):
        return v[:self.levels[l].r.n_owned_dofs]

    def _allreduce(self, t):
        self.dist.all_reduce(t)
        return t

    def dot(self, l, a, b):
        import torch
        s = torch.dot(self._owned(l, a).double(), self._owned(l, b).double()).reshape(1)
        return float(self._allreduce(s)[0])

    # ---- setup (PreconditionerGMG::initialize, main.cc:815-839)
    def interpolate(self, l, dst_coarse, src_fine):
        """interpolate_to_mg level l -> l-1 on owned + ghost coarse nodes."""
        self.levels[l].update_ghost_values(src_fine)
        self.tr.interpolate(l, dst_coarse, src_fine)
        self.levels[l - 1].update_ghost_values(dst_coarse)

    def set_linearization_point(self, params, u_fine, hist_fine=None, weights=None):
        """u_fine / hist_fine: finest-level local vectors in the level precision."""
        L = len(self.levels)
        us = [None] * L
        hs = [None] * L
        us[-1] = u_fine
        hs[-1] = hist_fine
        for l in range(L - 1, 0, -1):
            us[l - 1] = self.new_vector(l - 1)
            self.interpolate(l, us[l - 1], us[l])
            if hs[l] is not None:
                hs[l - 1] = []
                for h in hs[l]:
                    t = self.new_vector(l - 1)
                    self.interpolate(l, t, h)
                    hs[l - 1].append(t)
        self._lin0 = (params, us[0], hs[0], weights)
        for l, D in enumerate(self.levels):
            D.update_ghost_values(us[l])
            D.r.eng.set_parameters(**params)
            D.r.eng.set_linearization_point(us[l])
            if hs[l] is not None and params.get("order", 0) > 0:
                for h in hs[l]:
                    D.update_ghost_values(h)
                D.r.eng.set_previous_solution(hs[l], weights)

    def setup(self):
        for l, D in enumerate(self.levels):
            d = D.new_vector()
            D.r.eng.diagonal_raw(d)
            D.compress_add(d)
            D.r.eng.invert_diagonal(d)
            self.invdiag[l] = d
            if l == 0 and len(self.levels) > 1 and self.coarse_iters <= 0 and self.evs_levels <= 0:
                self.lam[l], self.omega[l] = 0.0, 1.0
                continue
            ev = 1.2 * self.power_iteration(l)
            self.lam[l] = ev
            alpha = ev / self.range if self.range > 1 else 0.9 * ev
            self.omega[l] = 2.0 / (alpha + ev) if ev > 0 else 1.0
        if self._coarse_direct:
            params, u0, h0, w = self._lin0
            D0 = self.levels[0]
            g = lambda v: D0.gather_global(v.to(D0.r.dtype))  # noqa: E731
            self.coarse.setup(params, g(u0), None if h0 is None else [g(h) for h in h0], w)

    def power_iteration(self, l):
        """deal.II power_iteration with set_initial_guess on the global dof
        index (x_i = i % 11 - mean, constrained 0), dots all-reduced."""
        import torch
        D = self.levels[l]
        n_glob = D.n_global_dofs
        mean = (n_glob // 11 * 55 + (n_glob % 11) * (n_glob % 11 - 1) // 2) / n_glob
        x = D.new_vector()
        xo = (self._global_dof[l] % 11).to(torch.float64) - mean
        con = D.r.con_owned
        xo[con] = 0.0
        x[:D.r.n_owned_dofs] = xo.to(x.dtype)

        # dots all-reduced on the device: no host round trip inside the
        # iteration, the estimate is read once at the end
        def ddot(a, b):
            t = torch.dot(self._owned(l, a).double(), self._owned(l, b).double()).reshape(1)
            return self._allreduce(t)

        x *= (1.0 / ddot(x, x).sqrt()).to(x.dtype)
        y = D.new_vector()
        lam = torch.zeros(1, dtype=torch.float64, device=x.device)
        d = self.invdiag[l]
        for _ in range(self.n_eig):
            D.vmult(y, x)
            y *= d
            lam = ddot(x, y)
            ny = ddot(y, y).sqrt()
            inv = torch.where(ny > 0, 1.0 / ny, torch.zeros_like(ny))
            x.copy_(y * inv.to(y.dtype))
        return abs(float(lam[0]))

    # ---- V-cycle (Multigrid::level_v_step)
    def relax(self, l, x, b, ax, zero):
        relax = getattr(self.tr, "relax", None)
        if relax is not None:
            return relax(l, x, b, ax, self.invdiag[l], self.omega[l], zero)
        w, d = self.omega[l], self.invdiag[l]
        if zero:
            x.copy_(w * d * b)
        else:
            x.add_(w * d * (b - ax))

    def smooth(self, l, x, b, zero, iters):
        D = self.levels[l]
        t = D.new_vector()
        it = 0
        if zero and iters > 0:
            self.relax(l, x, b, None, True)
            it = 1
        for _ in range(it, iters):
            D.vmult(t, x)
            self.relax(l, x, b, t, False)

    def v_step(self, l, x, b):
        if l == 0:
            if self._coarse_direct:
                D0 = self.levels[0]
                xg = self.coarse.solve(D0.gather_global(b))
                x.copy_(D0.scatter_global(xg).to(x.dtype))
            elif self.coarse_iters > 0:
                self.smooth(0, x, b, True, self.coarse_iters)
            else:
                x.copy_(b)
            return
        D, Dc = self.levels[l], self.levels[l - 1]
        self.smooth(l, x, b, True, self.n_smooth)
        t = D.new_vector()
        D.vmult(t, x)
        t.neg_().add_(b)
        bc = Dc.new_vector()
        self.tr.restrict_add(l, bc, t)
        Dc.compress_add(bc)
        xc = Dc.new_vector()
        self.v_step(l - 1, xc, bc)
        Dc.update_ghost_values(xc)
        self.tr.prolongate_add(l, x, xc)
        self.smooth(l, x, b, False, self.n_smooth)

    def vmult(self, dst, src):
        """PreconditionMG::vmult on finest-level local vectors (copy_to_mg /
        copy_from_mg convert to the level precision)."""
        L = len(self.levels) - 1
        D = self.levels[L]
        b = src.to(D.r.dtype)
        x = D.new_vector()
        self.v_step(L, x, b)
        dst.copy_(x.to(dst.dtype))
        return dst


def rank_child_lattices(meshes, parts_per_level, rank):
    """Rank-local child lattices (local fine node ids) with the global-first
    NOT_OWNER bits (bit 31) for every level pair, [None, l = 1, ...]."""
    out = [None]
    for l in range(1, len(meshes)):
        G = np.asarray(meshes[l - 1].child_lattice(meshes[l]), dtype=np.int64)
        own = global_first_owners(G)
        pc, pf = parts_per_level[l - 1][rank], parts_per_level[l][rank]
        g2l = np.full(meshes[l].n_nodes, -1, dtype=np.int64)
        g2l[pf.local_nodes] = np.arange(pf.n_nodes)
        loc = g2l[G[pc.cell_begin:pc.cell_end]]
        if (loc < 0).any():
            raise ValueError("a child lattice node is not local to the fine partition")
        ch = loc.astype(np.uint32)
        ch[~own[pc.cell_begin:pc.cell_end]] |= np.uint32(0x80000000)
        out.append(ch)
    return out


class NativeGroupMultigrid:
    """Every rank of a partitioned multigrid hierarchy in ONE process on one
    device (an in-process group), driven through the native team calls of
    the C-ABI (glsamd.PartitionedMultigrid: gls_dist_mg_* and
    gls_dist_gmres_solve, csrc/dist_mg.hip) — the single-GPU test of the
    distributed V-cycle and GMRES that RCCL ranks run one per GPU.  Levels on
    the same coarse-cell partition (main.cc:398-400); the FP64 outer operator
    on the finest level's partition."""

    def __init__(self, meshes, cmasks, world, precision="f32", coarse_n_iterations=10,
                 redundant_levels=0, **mg_kwargs):
        """redundant_levels = k > 0: level agglomeration (glsDistMGDesc
        n_redundant_levels): levels 0 .. k-1 and a copy of level k run
        single-domain on every rank, levels k .. are partitioned."""
        import glsamd
        self.world = world
        k = int(redundant_levels)
        n0 = meshes[0].n_cells
        cb = coarse_bounds(n0, world)
        all_parts = [build_partitions(m, world, [b * (m.n_cells // n0) for b in cb])
                     for m in meshes]
        self.parts, self.ranks, self.native = [], [], []
        for m, cm in zip(meshes[k:], cmasks[k:]):
            ratio = m.n_cells // n0
            parts = build_partitions(m, world, [b * ratio for b in cb])
            ranks = [RankOperator(m, cm, p, precision) for p in parts]
            nat = []
            for r in ranks:
                nat.append(r.eng.partitioned(r.part, group=nat[0] if nat else None))
            self.parts.append(parts)
            self.ranks.append(ranks)
            self.native.append(nat)
        fine_parts = build_partitions(meshes[-1], world,
                                      [b * (meshes[-1].n_cells // n0) for b in cb])
        self.fine = [RankOperator(meshes[-1], cmasks[-1], p, "f64") for p in fine_parts]
        self.fine_native = []
        for r in self.fine:
            self.fine_native.append(r.eng.partitioned(r.part, group=self.fine_native[0]
                                                      if self.fine_native else None))
        self.coarse_ops = [None] * world
        self.redundant_ops = [[] for _ in range(world)]
        redundant_child = None
        if coarse_n_iterations < 0 or k > 0:
            self.coarse_ops = [glsamd.NavierStokesOperator(meshes[k], cmasks[k], precision)
                               for _ in range(world)]
        if k > 0:
            self.redundant_ops = [[glsamd.NavierStokesOperator(meshes[l], cmasks[l], precision)
                                   for l in range(k)] for _ in range(world)]
            redundant_child = [None] + [meshes[l - 1].child_lattice(meshes[l])
                                        for l in range(1, k + 1)]
        nl = len(meshes) - k
        self.mg = []
        for r in range(world):
            child = rank_child_lattices(meshes, all_parts, r)
            child = [None] + child[k + 1:]
            self.mg.append(glsamd.PartitionedMultigrid(
                [self.native[l][r] for l in range(nl)], child,
                [self.parts[l][r].local_nodes[:self.parts[l][r].n_owned] for l in range(nl)],
                [m.n_nodes for m in meshes[k:]], coarse_n_iterations=coarse_n_iterations,
                coarse_global=self.coarse_ops[r],
                coarse_l2g=(self.parts[0][r].local_nodes
                            if coarse_n_iterations < 0 or k > 0 else None),
                redundant_ops=self.redundant_ops[r] or None, redundant_child=redundant_child,
                **mg_kwargs))

    def setup(self, params, u_star, hist=None, weights=None):
        """Parameters on every operator, the finest linearization point and
        history (replicated global arrays) scattered to the ranks, injected
        down the levels natively, then gls_dist_mg_setup; the FP64 outer
        operator gets the fine vectors directly."""
        import torch
        for ranks in self.ranks:
            for r in ranks:
                r.eng.set_parameters(**params)
        for op in self.coarse_ops:
            if op is not None:
                op.set_parameters(**params)
        for ops in self.redundant_ops:
            for op in ops:
                op.set_parameters(**params)
        fine = self.ranks[-1]
        u = [r.local_from_global(u_star) for r in fine]
        h = None
        if hist is not None and params.get("order", 0) > 0:
            h = [[r.local_from_global(x) for x in hist] for r in fine]
        glsamd_mg = type(self.mg[0])
        glsamd_mg.set_linearization_point(self.mg, u, h, weights)
        glsamd_mg.setup(self.mg)
        for r in self.fine:
            r.eng.set_parameters(**params)
            r.eng.set_linearization_point(r.local_from_global(u_star))
            if h is not None:
                r.eng.set_previous_solution([r.local_from_global(x) for x in hist], weights)
        torch.cuda.synchronize()

    def scatter(self, g, ranks=None):
        return [r.local_from_global(g) for r in (ranks or self.fine)]

    def gather(self, vs, ranks=None):
        import torch
        ranks = ranks or self.fine
        n = sum(r.n_owned_dofs for r in ranks)
        g = torch.zeros(n, dtype=vs[0].dtype, device=vs[0].device)
        for r, v in zip(ranks, vs):
            g.index_copy_(0, r.global_dofs[:r.n_owned_dofs], v[:r.n_owned_dofs])
        return g

    def vcycle(self, dsts, srcs):
        return type(self.mg[0]).vcycle(self.mg, dsts, srcs)

    def gmres(self, xs, bs, **kw):
        import glsamd
        return glsamd.dist_gmres_solve(self.fine_native, self.mg, xs, bs, **kw)

    # the same team calls made by one thread per member with n = 1 (the rank
    # code path of an RCCL rank; device copies as transport)
    def vcycle_threaded(self, dsts, srcs, reps=1):
        def one(r):
            for _ in range(reps):
                type(self.mg[r]).vcycle([self.mg[r]], [dsts[r]], [srcs[r]])
        run_threaded(self.world, one)

    def gmres_threaded(self, xs, bs, **kw):
        import glsamd
        return run_threaded(self.world, lambda r: glsamd.dist_gmres_solve(
            [self.fine_native[r]], [self.mg[r]], [xs[r]], [bs[r]], **kw))


class RedundantCoarseLU:
    """The deck's direct coarse solver for a partitioned hierarchy
    (multigrid.cc:448-455, 477-481): every rank holds the whole coarse level
    (400 cells at Re3900) as a single-domain operator and its dense LU
    (gls_mg with coarse_n_iterations = -1: rocSOLVER getrf + the inverse
    GEMV); the coarse right-hand side arrives all-gathered, the solution is
    sliced back to the rank's [owned | ghost] entries by the caller."""

    def __init__(self, mesh, cmask, precision):
        import glsamd
        self.op = glsamd.NavierStokesOperator(mesh, cmask, precision)
        self.mg = None
        self.precision = precision

    def setup(self, params, u, hist, weights):
        import glsamd
        import torch
        self.op.set_parameters(**params)
        self.op.set_linearization_point(u.to(self.op.dtype))
        if hist is not None and params.get("order", 0) > 0:
            self.op.set_previous_solution([h.to(self.op.dtype) for h in hist], weights)
        self.mg = glsamd.Multigrid([self.op], [], coarse_n_iterations=-1,
                                   outer_precision=self.precision)
        self.mg.setup()
        torch.cuda.synchronize()

    def solve(self, b):
        import torch
        x = torch.zeros_like(b)
        self.mg.vcycle(x, b)
        return x


class RedundantBottomMG:
    """Level agglomeration for the host-driven DistributedMultigrid (the
    native twin is glsDistMGDesc.n_redundant_levels): built over the global
    meshes 0 .. k and passed as the coarse_solver of a DistributedMultigrid
    over meshes k .. L with coarse_n_iterations = -1, it runs levels 0 .. k
    single-domain on every rank -- one V-cycle per coarse solve, the same
    smoother and the given coarse solver at the bottom -- after the level-k
    right-hand side arrives all-gathered.  Its linearization point and history
    are level k's, interpolated down the global levels (build_gmg).  The
    V-cycle of the whole hierarchy, with the small levels' halo exchanges
    replaced by one gather (deal.II re-partitions such levels instead,
    main.cc:398-400)."""

    def __init__(self, meshes, cmasks, precision, coarse_n_iterations=10, **mg_kwargs):
        self.meshes, self.cmasks, self.precision = list(meshes), list(cmasks), precision
        self.coarse_n_iterations, self.mg_kwargs = coarse_n_iterations, mg_kwargs
        self.mg = self.ops = None

    def __call__(self, mesh, cmask, precision):
        # the coarse_solver factory protocol: level 0 of the partitioned
        # hierarchy must be this bottom's finest level
        if mesh.n_cells != self.meshes[-1].n_cells or precision != self.precision:
            raise ValueError("RedundantBottomMG: the partitioned hierarchy must start at the "
                             "bottom's finest level, in its precision")
        return self

    def setup(self, params, u, hist, weights):
        import glsamd
        import torch
        h = None if hist is None or params.get("order", 0) == 0 else list(hist)
        self.mg, self.ops = glsamd.build_gmg(self.meshes, self.cmasks, params, u, h, weights,
                                             precision=self.precision,
                                             coarse_n_iterations=self.coarse_n_iterations,
                                             outer_precision=self.precision, **self.mg_kwargs)
        torch.cuda.synchronize()

    def solve(self, b):
        import torch
        x = torch.zeros_like(b)
        self.mg.vcycle(x, b)
        return x


def gmres_solve(apply_A, apply_P, b, x, n_owned, allreduce, max_n_tmp_vectors=30,
                max_iterations=10000, relative_tolerance=1e-8, absolute_tolerance=1e-12):
    """LinearSolverGMRES::solve (solver_l.cc:45-74) on rank-local vectors of a
    partitioned operator: right-preconditioned restarted GMRES(m = 28) with
    classical Gram-Schmidt + one re-orthogonalisation, the basis V in HBM,
    dots over the owned entries all-reduced (MPI_Allreduce in deal.II;
    RCCL / gloo here).  x = 0 on entry; returns (iterations, residual);
    raises RuntimeError on no convergence (SolverControl::NoConvergence)."""
    import torch
    m = max_n_tmp_vectors - 2
    n = b.numel()
    dev, dt = b.device, torch.float64

    def ared(t):
        allreduce(t)
        return t

    def nrm(v):
        return float(ared((v[:n_owned].double() ** 2).sum().reshape(1))[0]) ** 0.5

    bnorm = nrm(b)
    tol = max(relative_tolerance * bnorm, absolute_tolerance)
    x.zero_()
    V = torch.zeros(m + 1, n, dtype=b.dtype, device=dev)
    z = torch.zeros_like(b)
    w = torch.zeros_like(b)
    it, res = 0, bnorm
    V[0].copy_(b)
    while res > tol and it < max_iterations:
        beta = res
        V[0] *= 1.0 / beta
        H = np.zeros((m + 1, m))
        g = np.zeros(m + 1)
        g[0] = beta
        cs, sn = np.zeros(m), np.zeros(m)
        jd = 0
        for j in range(m):
            if it >= max_iterations:
                break
            apply_P(z, V[j])
            apply_A(w, z)
            hj = torch.zeros(j + 1, dtype=dt, device=dev)
            for _ in range(2):
                h = ared(V[:j + 1, :n_owned].double() @ w[:n_owned].double())
                w.sub_((h.to(w.dtype) @ V[:j + 1]))
                hj += h
            # the Hessenberg column and the new norm cross to the host together
            hn2 = ared((w[:n_owned].double() ** 2).sum().reshape(1))
            col = torch.cat([hj, hn2]).cpu().numpy()
            hn = float(col[j + 1]) ** 0.5
            H[:j + 1, j] = col[:j + 1]
            H[j + 1, j] = hn
            if hn > 0:
                V[j + 1].copy_(w * (1.0 / hn))
            for i in range(j):
                tmp = cs[i] * H[i, j] + sn[i] * H[i + 1, j]
                H[i + 1, j] = -sn[i] * H[i, j] + cs[i] * H[i + 1, j]
                H[i, j] = tmp
            rr = np.hypot(H[j, j], H[j + 1, j])
            cs[j] = H[j, j] / rr if rr > 0 else 1.0
            sn[j] = H[j + 1, j] / rr if rr > 0 else 0.0
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
        w.copy_(torch.from_numpy(y).to(device=dev, dtype=b.dtype) @ V[:jd])
        apply_P(z, w)
        x.add_(z)
        if res <= tol or it >= max_iterations:
            break
        apply_A(V[0], x)
        V[0].neg_().add_(b)
        res = nrm(V[0])
    if res > tol:
        raise RuntimeError(f"GMRES: no convergence in {it} iterations ({res} > {tol})")
    return it, res
