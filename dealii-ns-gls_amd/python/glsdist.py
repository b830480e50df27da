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


def build_partitions(mesh, world):
    """Split the cell list into `world` contiguous brick ranges and derive the
    ownership / ghost / exchange plan for every rank."""
    nbc = _brick_cells(mesh)
    if mesh.n_cells % nbc:
        raise ValueError("cell count is not a multiple of the brick size")
    nb = mesh.n_cells // nbc
    if world > nb:
        raise ValueError(f"{world} ranks for {nb} bricks")
    bounds = [(r * nb // world) * nbc for r in range(world + 1)]
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
        self._brick = mesh.brick()

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

    def __init__(self, mesh, cmask, precision, dist, rank, world, engine="gpu", native=None):
        self.dist, self.rank, self.world = dist, rank, world
        self.parts = build_partitions(mesh, world)
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
        sends, recvs = self.r.pack_import(v)
        self._exchange(sends, recvs)
        self.r.unpack_import(v)

    def compress_add(self, v):
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
