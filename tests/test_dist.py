"""Partitioned (multi-GPU) operator path: partition plan, ghost exchange and
the distributed vmult (glsdist.py).

CPU tests run the same per-rank phases with the oracle as the local operator
(TEST INFRASTRUCTURE engine) — in-process over several ranks and over a real
world_size-2 gloo process group; the GPU test runs the product local
operator (libglsamd.so) for 2 and 4 partitions on one device.  All compare
against the single-domain oracle vmult on the same inputs (FP64: 1e-12)."""
import os

import numpy as np
import pytest

import glsdist
from dist_engines import OracleEngine
from helpers import deck_case, rel_err

CASES = [("input_hoffmann_3D_Re3900.json", 1), ("input_turek_2D_Re100.json", 2)]


@pytest.mark.parametrize("name,n_ref", CASES)
@pytest.mark.parametrize("world", [2, 3, 5])
def test_partition_plan(name, n_ref, world):
    c = deck_case(name, n_ref)
    m = c.mesh
    parts = glsdist.build_partitions(m, world)
    # cells: contiguous, complete, brick aligned
    assert parts[0].cell_begin == 0 and parts[-1].cell_end == m.n_cells
    nbc = int(np.prod([max(1, b) for b in m.brick()[:m.dim]]))
    for a, b in zip(parts, parts[1:]):
        assert a.cell_end == b.cell_begin and a.cell_end % nbc == 0
    # every node owned exactly once
    owned = np.concatenate([p.local_nodes[:p.n_owned] for p in parts])
    assert np.array_equal(np.sort(owned), np.arange(m.n_nodes))
    for p in parts:
        # every local node is touched by a local cell and vice versa
        touched = np.unique(m.cell_nodes[p.cell_begin:p.cell_end])
        assert np.array_equal(np.sort(p.local_nodes), touched)
        # ghosts are owned by a lower-or-higher rank that also touches them
        assert np.all(p.node_owner[:p.n_owned] == p.rank)
        assert np.all(p.node_owner[p.n_owned:] != p.rank)
        for q, recv in p.recv_nodes.items():
            send = parts[q].send_nodes[p.rank]
            assert np.array_equal(p.local_nodes[recv], parts[q].local_nodes[send])


def _oracle_ref(c):
    return c.oracle().vmult(c.src)


@pytest.mark.parametrize("name,n_ref", CASES)
@pytest.mark.parametrize("world", [1, 2, 4])
def test_local_group_oracle(name, n_ref, world):
    import torch
    c = deck_case(name, n_ref)
    g = glsdist.LocalGroup(c.mesh, c.cmask, world, engine=OracleEngine)
    g.setup(c.params, c.u_star, c.hist, c.weights)
    srcs = g.scatter(c.src)
    dsts = [r.new_vector() for r in g.ranks]
    g.vmult(dsts, srcs)
    out = g.gather(dsts).numpy()
    assert rel_err(out, _oracle_ref(c)) < 1e-12
    # src ghosts were imported bit-exactly from their owners
    for r, s in zip(g.ranks, srcs):
        assert torch.equal(s, torch.from_numpy(c.src)[r.global_dofs])


def _gloo_worker(rank, world, port, name, n_ref, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "dealii-ns-gls_amd", "python"), os.path.join(root, "oracle"),
              os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import glsdist as gd
    from helpers import deck_case as dc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = dc(name, n_ref)
        op = gd.DistributedOperator(c.mesh, c.cmask, "f64", dist, rank, world, engine=OracleEngine)
        op.setup(c.params, c.u_star, c.hist, c.weights)
        src = op.scatter_global(c.src)
        src[op.r.n_owned_dofs:].zero_()  # ghosts must come from the exchange
        dst = op.new_vector()
        op.vmult(dst, src)
        g = op.gather_global(dst)
        if rank == 0:
            q.put(g.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,n_ref", CASES + [("input_sphere_amg.json", 1)])
def test_gloo_world2(name, n_ref):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, name, n_ref, q))
             for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = deck_case(name, n_ref)
    assert rel_err(out, _oracle_ref(c)) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_ref", CASES)
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("native", [False, True])
def test_local_group_gpu(name, n_ref, world, native):
    """native: libglsamd's gls_dist phases (pack, interior bricks, import,
    boundary bricks + reduce, export, unpack-add) with in-process copies in
    place of RCCL; otherwise the torch-side exchange around gls_op_vmult."""
    import torch
    c = deck_case(name, n_ref)
    g = glsdist.LocalGroup(c.mesh, c.cmask, world, engine="gpu", native=native)
    g.setup(c.params, c.u_star, c.hist, c.weights)
    srcs = g.scatter(c.src)
    dsts = [r.new_vector() for r in g.ranks]
    if native:
        for r, sv in zip(g.ranks, srcs):  # ghosts must come from the import
            sv[r.n_owned_dofs:].zero_()
    g.vmult(dsts, srcs)
    torch.cuda.synchronize()
    out = g.gather(dsts).cpu().numpy()
    assert rel_err(out, _oracle_ref(c)) < 1e-12
    if native:
        for r, sv, dv in zip(g.ranks, srcs, dsts):
            assert torch.equal(sv.cpu(), torch.from_numpy(c.src)[r.global_dofs.cpu()])
            assert not dv[r.n_owned_dofs:].any()  # compress zeroes the ghosts
        n_int = [m.interior_bricks() for m in g.native]
        assert all(0 <= a <= b for a, b in n_int)
        if world == 2 and name.startswith("input_hoffmann"):
            assert all(a > 0 for a, _ in n_int)  # something to overlap with


@pytest.mark.gpu
def test_rccl_world1_native():
    """The RCCL path end to end on one GPU: torch.distributed (nccl = RCCL)
    world 1, the RCCL unique id broadcast, ncclCommInitRank inside
    libglsamd, gls_dist_vmult (pack / interior / event wait / boundary /
    reduce / export / unpack with no peers) against gls_op_vmult."""
    import socket
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        c = deck_case("input_hoffmann_3D_Re3900.json", 1)
        op = glsdist.DistributedOperator(c.mesh, c.cmask, "f64", dist, 0, 1)
        assert op.native is not None
        op.setup(c.params, c.u_star, c.hist, c.weights)
        src = op.scatter_global(c.src)
        dst = op.new_vector()
        op.vmult(dst, src)
        ref = op.new_vector()
        op.op.vmult(ref, src)
        torch.cuda.synchronize()
        # equal up to the LDS-atomic summation order of the brick kernel
        assert rel_err(dst.cpu().numpy(), ref.cpu().numpy()) < 1e-14
        assert rel_err(dst.cpu().numpy(), _oracle_ref(c)) < 1e-12
    finally:
        dist.destroy_process_group()


def test_sphere_r3_partition_balance():
    """BASELINE's sphere configuration (input_sphere_amg.json r3, 524,288
    unstructured cells, "load balance at 8 GPUs"): the 8-rank partition gives
    every rank the same cells, owned nodes within 5 % of the mean, ghosts
    below 10 % of the owned nodes and at most two peers per rank."""
    from helpers import deck
    m = deck("input_sphere_amg.json").mesh(3)
    parts = glsdist.build_partitions(m, 8)
    cells = [p.cell_end - p.cell_begin for p in parts]
    owned = np.array([p.n_owned for p in parts])
    ghost = np.array([p.n_nodes - p.n_owned for p in parts])
    assert len(set(cells)) == 1 and sum(cells) == m.n_cells
    assert np.abs(owned / owned.mean() - 1).max() < 0.05
    assert (ghost < 0.10 * owned).all()
    assert max(len(p.recv_nodes) for p in parts) <= 2


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_local_group_gpu_two_layer(world, monkeypatch):
    """The partitioned native vmult with two-layer bricks forced
    (GLS_TWO_LAYER=1: 4x4x2 bricks, the default only from 8 dispatch
    generations, e.g. a rank's r3 slab at 2 ranks): interior / boundary
    segments, curved-brick balance and the ghost-row reduce on 32-cell
    bricks, against the single-domain oracle (FP64 1e-12)."""
    import torch
    monkeypatch.setenv("GLS_TWO_LAYER", "1")
    c = deck_case("input_hoffmann_3D_Re3900.json", 1)
    g = glsdist.LocalGroup(c.mesh, c.cmask, world, engine="gpu", native=True)
    g.setup(c.params, c.u_star, c.hist, c.weights)
    assert all(list(r.eng.op.brick_shape)[2] == 2 for r in g.ranks), \
        [list(r.eng.op.brick_shape) for r in g.ranks]
    srcs = g.scatter(c.src)
    dsts = [r.new_vector() for r in g.ranks]
    for r, sv in zip(g.ranks, srcs):  # ghosts must come from the import
        sv[r.n_owned_dofs:].zero_()
    g.vmult(dsts, srcs)
    torch.cuda.synchronize()
    out = g.gather(dsts).cpu().numpy()
    assert rel_err(out, _oracle_ref(c)) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_ref", CASES)
@pytest.mark.parametrize("world", [2, 4])
def test_threaded_group_vmult(name, n_ref, world):
    """gls_dist_vmult itself — the production schedule of an RCCL rank: pack,
    import on the communication stream || first interior half, boundary
    bricks + ghost-row reduce after the import event, export on the
    communication stream || second interior half + owned-row reduce, unpack
    after the export event — with one host thread and one stream pair per
    member of an in-process group (device copies gated by the peers' events
    as transport, csrc/dist.hip GroupTransport), three times back to back
    (the send-buffer and ghost-row fences between calls), against the
    single-domain oracle (FP64 1e-12)."""
    import torch
    c = deck_case(name, n_ref)
    g = glsdist.LocalGroup(c.mesh, c.cmask, world, engine="gpu", native=True)
    g.setup(c.params, c.u_star, c.hist, c.weights)
    srcs = g.scatter(c.src)
    dsts = [r.new_vector() for r in g.ranks]
    for r, sv in zip(g.ranks, srcs):  # ghosts must come from the import
        sv[r.n_owned_dofs:].zero_()
    for dv in dsts:
        dv.fill_(7.0)
    g.vmult_threaded(dsts, srcs, reps=3)
    torch.cuda.synchronize()
    out = g.gather(dsts).cpu().numpy()
    assert rel_err(out, _oracle_ref(c)) < 1e-12
    for r, sv, dv in zip(g.ranks, srcs, dsts):
        assert torch.equal(sv.cpu(), torch.from_numpy(c.src)[r.global_dofs.cpu()])
        assert not dv[r.n_owned_dofs:].any()  # compress zeroes the ghosts
