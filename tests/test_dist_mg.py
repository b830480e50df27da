"""Multi-GPU on the preconditioner side: the
partitioned multigrid (per-level partitions on the same coarse cells,
main.cc:398-400; halo exchanges around the transfers, main.cc:540-563) and
GMRES with all-reduced dots (solver_l.cc:45-74), glsdist.DistributedMultigrid
/ gmres_solve, against the single-domain restatement on the same inputs.

CPU: world_size-2 gloo process group, the oracle as every rank's local
operator (tests/dist_engines.py); FP64 throughout, so the partitioned V-cycle
and GMRES solution agree with the single-domain ones to 1e-10 (summation
order only).  GPU: the product path (libglsamd.so kernels, RCCL exchange) at
world 1 against the single-domain GPU multigrid."""
import os

import numpy as np
import pytest

import glsdist
from helpers import deck, rel_err

CASE = ("input_hoffmann_3D_Re3900.json", 1)
# a short solve (GMRES(28), a few dozen iterations) keeps the CPU test brief
GMRES_TOL = 1e-3
GMRES_M = 30


def _hierarchy(name, n_ref):
    import glsinputs as gi
    d = deck(name)
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    b = gi.rnd(11, meshes[-1].n_dofs)
    return meshes, cm, params, w, u, hist, b


def _single_domain(name, n_ref, coarse):
    """OracleGMG V-cycle and GMRES(OracleGMG) with the oracle operator."""
    import torch
    import oracle as orc
    from mg_ref import OracleGMG
    meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=coarse)
    ref.setup_omega()
    o = orc.Oracle(orc.OracleMesh(meshes[-1], cm[-1]), **params)
    o.set_linearization_point(u)
    o.set_previous_solution(hist, w)
    vc = ref.vcycle(b)
    if coarse == 0:
        return ref.omega, vc, None, 0
    x = torch.zeros(len(b), dtype=torch.float64)
    bt = torch.from_numpy(b)
    it, res = glsdist.gmres_solve(
        lambda dst, src: dst.copy_(torch.from_numpy(o.vmult(src.numpy()))),
        lambda dst, src: dst.copy_(torch.from_numpy(ref.vcycle(src.numpy()))),
        bt, x, len(b), lambda t: t, relative_tolerance=GMRES_TOL,
        max_n_tmp_vectors=GMRES_M)
    return ref.omega, vc, x.numpy(), it


def _worker(rank, world, port, name, n_ref, coarse, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "dealii-ns-gls_amd", "python"), os.path.join(root, "oracle"),
              os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import glsdist as gd
    from dist_engines import OracleEngine, OracleTransfers
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)
        dmg = gd.DistributedMultigrid(meshes, cm, "f64", dist, rank, world, engine=OracleEngine,
                                      transfers=lambda m: OracleTransfers(m, meshes),
                                      coarse_n_iterations=coarse)
        top = dmg.levels[-1]
        dmg.set_linearization_point(params, top.scatter_global(u),
                                    [top.scatter_global(h) for h in hist], w)
        dmg.setup()
        bl = top.scatter_global(b)
        xl = top.new_vector()
        dmg.vmult(xl, bl)
        vc = top.gather_global(xl).numpy()
        if coarse == 0:  # V-cycle only
            if rank == 0:
                q.put((list(dmg.omega), vc, None, 0))
            return
        # the fine FP64 operator on the finest level's partition
        A = dmg.fine_operator("f64")
        A.setup(params, u, hist, w)
        x = A.new_vector()
        it, res = gd.gmres_solve(lambda dst, src: A.vmult(dst, src),
                                 lambda dst, src: dmg.vmult(dst, src),
                                 A.scatter_global(b), x, A.r.n_owned_dofs,
                                 lambda t: dist.all_reduce(t), relative_tolerance=GMRES_TOL,
        max_n_tmp_vectors=GMRES_M)
        xs = A.gather_global(x).numpy()
        if rank == 0:
            q.put((list(dmg.omega), vc, xs, it))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("coarse", [10, 0])
def test_gloo_world2_vcycle_gmres(coarse):
    import socket
    import torch.multiprocessing as mp
    name, n_ref = CASE
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, n_ref, coarse, q))
             for r in range(2)]
    for p in procs:
        p.start()
    # the single-domain reference runs while the ranks work
    omega_ref, vc_ref, xs_ref, it_ref = _single_domain(name, n_ref, coarse)
    omega, vc, xs, it = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for l, (a, r) in enumerate(zip(omega, omega_ref)):
        if l == 0 and coarse <= 0:
            continue
        assert abs(a - r) < 1e-10 * r, (l, a, r)
    assert rel_err(vc, vc_ref) < 1e-10
    if xs is not None:
        assert abs(it - it_ref) <= 1
        assert rel_err(xs, xs_ref) < 1e-7


@pytest.mark.gpu
def test_rccl_world1_multigrid_gmres():
    """The product path of the partitioned multigrid at world 1 (RCCL
    communicator, libglsamd.so transfers / diagonals / relaxation kernels)
    against the single-domain GPU multigrid and GMRES."""
    import torch
    import torch.distributed as dist
    import glsamd
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        name, n_ref = CASE
        meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)
        dmg = glsdist.DistributedMultigrid(meshes, cm, "f32", dist, 0, 1, coarse_n_iterations=10)
        top = dmg.levels[-1]
        dmg.set_linearization_point(params, top.scatter_global(u),
                                    [top.scatter_global(h) for h in hist], w)
        dmg.setup()
        mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                                   coarse_n_iterations=10)
        for l in range(len(meshes)):
            wd, lam = mg.relaxation(l)
            assert abs(dmg.omega[l] - wd) < 1e-4 * wd, (l, dmg.omega[l], wd)
        bd = torch.from_numpy(b).cuda()
        x1 = torch.zeros_like(bd)
        dmg.vmult(x1, top.scatter_global(b).double())
        x2 = torch.zeros_like(bd)
        mg.vcycle(x2, bd)
        torch.cuda.synchronize()
        g1 = top.gather_global(x1).cpu().numpy()
        assert rel_err(g1, x2.cpu().numpy()) < 1e-3  # FP32 levels, different omega rounding
        A = dmg.fine_operator("f64")
        A.setup(params, u, hist, w)
        x = A.new_vector()
        it, res = glsdist.gmres_solve(lambda dst, src: A.vmult(dst, src),
                                      lambda dst, src: dmg.vmult(dst, src),
                                      A.scatter_global(b), x, A.r.n_owned_dofs,
                                      lambda t: dist.all_reduce(t), relative_tolerance=1e-6)
        Ad = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
        Ad.set_parameters(**params)
        Ad.set_linearization_point(u)
        Ad.set_previous_solution(hist, w)
        lin = glsamd.LinearSolverGMRES(Ad, mg, relative_tolerance=1e-6)
        xd = Ad.initialize_dof_vector()
        lin.solve(xd, bd)
        torch.cuda.synchronize()
        assert abs(it - lin.last["n_iterations"]) <= 2, (it, lin.last)
        assert rel_err(A.gather_global(x).cpu().numpy(), xd.cpu().numpy()) < 1e-4
    finally:
        dist.destroy_process_group()


def _worker_direct(rank, world, port, name, n_ref, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "dealii-ns-gls_amd", "python"), os.path.join(root, "oracle"),
              os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import glsdist as gd
    from dist_engines import OracleCoarseDirect, OracleEngine, OracleTransfers
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)
        dmg = gd.DistributedMultigrid(meshes, cm, "f64", dist, rank, world, engine=OracleEngine,
                                      transfers=lambda m: OracleTransfers(m, meshes),
                                      coarse_n_iterations=-1, coarse_solver=OracleCoarseDirect)
        top = dmg.levels[-1]
        dmg.set_linearization_point(params, top.scatter_global(u),
                                    [top.scatter_global(h) for h in hist], w)
        dmg.setup()
        xl = top.new_vector()
        dmg.vmult(xl, top.scatter_global(b))
        vc = top.gather_global(xl).numpy()
        if rank == 0:
            q.put((list(dmg.omega), vc))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_vcycle_direct_coarse():
    """The deck's direct coarse solver on a partitioned hierarchy: the coarse
    right-hand side all-gathered, solved redundantly on every rank
    (glsdist.RedundantCoarseLU on the GPU; the oracle's dense solve here)."""
    import socket
    import torch.multiprocessing as mp
    from mg_ref import OracleGMG
    name, n_ref = "input_turek_2D_Re100.json", 1
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_direct, args=(r, 2, port, name, n_ref, q))
             for r in range(2)]
    for p in procs:
        p.start()
    meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=-1)
    ref.setup_omega()
    vc_ref = ref.vcycle(b)
    omega, vc = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert abs(omega[1] - ref.omega[1]) < 1e-10 * ref.omega[1]
    assert rel_err(vc, vc_ref) < 1e-10


@pytest.mark.gpu
def test_rccl_world1_direct_coarse():
    """The partitioned multigrid with the deck's direct coarse solver
    (glsdist.RedundantCoarseLU: the coarse level and its dense LU on every
    rank) at world 1 over RCCL, against the single-domain GPU multigrid with
    the same coarse solver."""
    import torch
    import torch.distributed as dist
    import glsamd
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        meshes, cm, params, w, u, hist, b = _hierarchy(*CASE)
        dmg = glsdist.DistributedMultigrid(meshes, cm, "f32", dist, 0, 1, coarse_n_iterations=-1)
        top = dmg.levels[-1]
        dmg.set_linearization_point(params, top.scatter_global(u),
                                    [top.scatter_global(h) for h in hist], w)
        dmg.setup()
        mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                                   coarse_n_iterations=-1)
        bd = torch.from_numpy(b).cuda()
        x1 = torch.zeros_like(bd)
        dmg.vmult(x1, top.scatter_global(b).double())
        x2 = torch.zeros_like(bd)
        mg.vcycle(x2, bd)
        torch.cuda.synchronize()
        assert rel_err(top.gather_global(x1).cpu().numpy(), x2.cpu().numpy()) < 1e-3
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_native_mg_plan(world):
    """The per-rank plan of the native partitioned multigrid
    (glsdist.rank_child_lattices -> gls_dist_mg_create): on every level pair
    each global fine node is claimed (NOT_OWNER bit clear) by exactly one
    (rank, coarse cell) lattice entry, and that rank owns the node in the
    fine partition — the invariant the owner-only restriction and
    prolongation rely on (every owned fine row is written / read by its own
    rank only)."""
    from helpers import deck
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(2)]
    n0 = meshes[0].n_cells
    cb = glsdist.coarse_bounds(n0, world)
    parts = [glsdist.build_partitions(m, world, [b * (m.n_cells // n0) for b in cb])
             for m in meshes]
    claims = np.zeros(meshes[1].n_nodes, dtype=np.int64)
    for r in range(world):
        ch = glsdist.rank_child_lattices(meshes, parts, r)[1]
        pf = parts[1][r]
        own = (ch & np.uint32(0x80000000)) == 0
        loc = (ch & np.uint32(0x7FFFFFFF)).astype(np.int64)
        assert (loc < pf.n_nodes).all()
        gl = pf.local_nodes[loc[own]]
        np.add.at(claims, gl, 1)
        # the claiming rank owns the node (local index in the owned prefix)
        assert (loc[own] < pf.n_owned).all()
    assert (claims == 1).all()


def _worker_agglomerated(rank, world, port, name, n_ref, k, q):
    """A rank of the host-driven partitioned multigrid with level agglomeration
    (glsdist.RedundantBottomMG's protocol): levels k .. partitioned, levels
    0 .. k single-domain on every rank behind one gather (here an oracle
    multigrid as the bottom, the CPU engine of the tests)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "dealii-ns-gls_amd", "python"), os.path.join(root, "oracle"),
              os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import glsdist as gd
    from dist_engines import OracleEngine, OracleTransfers
    from mg_ref import OracleGMG
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)

        class OracleBottom:
            def __call__(self, mesh, cmask, precision):
                return self

            def setup(self, prm, u0, h0, wts):
                self.g = OracleGMG(meshes[:k + 1], cm[:k + 1], prm, u0.numpy(),
                                   None if h0 is None else [h.numpy() for h in h0], wts,
                                   coarse_iters=10)
                self.g.setup_omega()

            def solve(self, rhs):
                return torch.from_numpy(self.g.vcycle(rhs.double().numpy()))

        dmg = gd.DistributedMultigrid(meshes[k:], cm[k:], "f64", dist, rank, world,
                                      engine=OracleEngine,
                                      transfers=lambda m: OracleTransfers(m, meshes[k:]),
                                      coarse_n_iterations=-1, coarse_solver=OracleBottom())
        top = dmg.levels[-1]
        dmg.set_linearization_point(params, top.scatter_global(u),
                                    [top.scatter_global(h) for h in hist], w)
        dmg.setup()
        bl = top.scatter_global(b)
        xl = top.new_vector()
        dmg.vmult(xl, bl)
        vc = top.gather_global(xl).numpy()
        if rank == 0:
            q.put((list(dmg.omega), vc))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_vcycle_agglomerated():
    """Level agglomeration on the host-driven path at world size 2 (gloo, the
    oracle as every rank's operator): 2D Turek Re100 r0..r2 with r2
    partitioned and r0, r1 single-domain on every rank (the coarse_solver
    protocol glsdist.RedundantBottomMG implements on the GPU) -- the V-cycle
    of the single-domain three-level hierarchy to 1e-10, the partitioned
    level's relaxation factor to 1e-10 (the native
    twin: tests/test_gpu_dist_native.py::test_native_group_vcycle_agglomerated)."""
    import socket
    import torch.multiprocessing as mp
    from mg_ref import OracleGMG
    name, n_ref, k = "input_turek_2D_Re100.json", 2, 1
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_agglomerated, args=(r, 2, port, name, n_ref, k, q))
             for r in range(2)]
    for p in procs:
        p.start()
    meshes, cm, params, w, u, hist, b = _hierarchy(name, n_ref)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=10)
    ref.setup_omega()
    vc_ref = ref.vcycle(b)
    omega, vc = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert abs(omega[-1] - ref.omega[-1]) < 1e-10 * ref.omega[-1], (omega, ref.omega)
    err = rel_err(vc, vc_ref)
    print(f"gloo world 2, {k + 1} of {n_ref + 1} levels agglomerated: V-cycle vs single-domain "
          f"{err:.2e}")
    assert err < 1e-10


@pytest.mark.gpu
def test_rccl_world1_agglomerated_bottom():
    """glsdist.RedundantBottomMG on the product path at world 1 (RCCL): the
    host-driven partitioned multigrid over Re3900 r1..r2 whose coarse solve is
    the single-domain r0..r1 V-cycle on every rank, against the single-domain
    r0..r2 GPU V-cycle (FP32 levels)."""
    import torch
    import torch.distributed as dist
    import glsamd
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        meshes, cm, params, w, u, hist, b = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
        bottom = glsdist.RedundantBottomMG(meshes[:2], cm[:2], "f32", coarse_n_iterations=10)
        dmg = glsdist.DistributedMultigrid(meshes[1:], cm[1:], "f32", dist, 0, 1,
                                           coarse_n_iterations=-1, coarse_solver=bottom)
        top = dmg.levels[-1]
        dmg.set_linearization_point(params, top.scatter_global(u),
                                    [top.scatter_global(h) for h in hist], w)
        dmg.setup()
        mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                                   coarse_n_iterations=10)
        wd, lam = mg.relaxation(2)
        assert abs(dmg.omega[-1] - wd) < 1e-4 * wd, (dmg.omega, wd)
        bd = torch.from_numpy(b).cuda()
        x1 = torch.zeros_like(bd)
        dmg.vmult(x1, top.scatter_global(b).double())
        x2 = torch.zeros_like(bd)
        mg.vcycle(x2, bd)
        torch.cuda.synchronize()
        err = rel_err(top.gather_global(x1).cpu().numpy(), x2.cpu().numpy())
        print(f"world 1 host-driven, r0..r1 agglomerated: V-cycle vs single-domain {err:.2e}")
        assert err < 1e-3  # FP32 levels, different omega rounding (as the test above)
    finally:
        dist.destroy_process_group()
