"""Brick discovery for an arbitrary cell order (csrc/brick_discovery.cc,
VERDICT r1 item 6): a deal.II mesh arrives in MatrixFree's cell order, not
the generator's brick order; gls_op_create(brick = {-1,-1,-1}) finds the
structured blocks from the connectivity and runs the brick kernel on them.

CPU: the discovery itself (gls_discover_bricks, host only) on shuffled /
re-oriented meshes — the shape it must find and a valid tiling.  GPU: the
operator on those meshes against the oracle on the same mesh (FP64 1e-12,
FP32 2e-5) and the multigrid over shuffled levels."""
import numpy as np
import pytest

import glsinputs as gi
from helpers import Case, deck, rel_err
from shuffle import ShuffledMesh, check_tiling

RE3900 = "input_hoffmann_3D_Re3900.json"


def _case(mesh, name):
    d = deck(name)
    vel, p, slip = d.boundary_descriptor()
    params, w = d.operator_parameters(2.5e-4)
    return Case(mesh, mesh.constraint_mask(vel, p, slip), params, w, u_inf=d.u_max)


@pytest.mark.parametrize("name,n_ref,expect", [
    (RE3900, 2, (4, 4, 1)), (RE3900, 1, (2, 2, 2)), ("input_turek_2D_Re100.json", 3, (8, 8, 1)),
    ("input_turek_3D_Re100.json", 2, (4, 4, 1))])
def test_discovery_shuffled(name, n_ref, expect):
    import glsamd
    m = deck(name).mesh(n_ref)
    for mesh in (m, ShuffledMesh(m, seed=n_ref)):
        shape, perm = glsamd.discover_bricks(mesh)
        assert shape == expect, shape
        check_tiling(mesh.cell_nodes, mesh.dim, mesh.degree, shape, perm)


@pytest.mark.parametrize("name,n_ref", [(RE3900, 1), ("input_turek_2D_Re20_stat.json", 2)])
def test_discovery_reoriented(name, n_ref):
    """Randomly rotated cell numberings break the blocks: whatever is found
    (down to single cells) must still tile."""
    import glsamd
    mesh = ShuffledMesh(deck(name).mesh(n_ref), seed=7, rotate=True)
    shape, perm = glsamd.discover_bricks(mesh)
    assert shape != (0, 0, 0)
    check_tiling(mesh.cell_nodes, mesh.dim, mesh.degree, shape, perm)


def test_discovery_sphere():
    import glsamd
    import glsmesh as gm
    d = gm.read_deck(f"{gm.DECK_DIR}/input_sphere_amg.json")
    m = d.mesh(1)
    shape, perm = glsamd.discover_bricks(ShuffledMesh(m, seed=3))
    assert shape == (2, 2, 2)
    check_tiling(ShuffledMesh(m, seed=3).cell_nodes, 3, m.degree, shape, perm)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_ref,rotate,prec", [
    (RE3900, 2, False, "f64"), (RE3900, 2, False, "f32"), (RE3900, 1, True, "f64"),
    ("input_turek_2D_Re100.json", 3, False, "f64")])
def test_gpu_vmult_shuffled(name, n_ref, rotate, prec):
    import torch
    mesh = ShuffledMesh(deck(name).mesh(n_ref), seed=11, rotate=rotate)
    case = _case(mesh, name)
    op = case.gpu(prec)
    if not rotate:
        assert op.brick_shape != (0, 0, 0)
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.u_star))
    torch.cuda.synchronize()
    o = case.oracle()
    tol = 1e-12 if prec == "f64" else 2e-5
    assert rel_err(dst.double().cpu().numpy(), o.vmult(case.src)) < tol
    assert rel_err(res.double().cpu().numpy(), o.evaluate_residual(case.u_star)) < tol
    # tables round trip in the caller's cell order
    t_gpu = op.download_tables()[0]
    t_ref = o.tables()[0]
    assert rel_err(t_gpu, t_ref) < (1e-12 if prec == "f64" else 1e-6)


@pytest.mark.gpu
def test_gpu_vcycle_shuffled_levels():
    """The multigrid over shuffled levels (child lattices in the caller's
    cell order, the coarse operators' discovered order inside) against the
    oracle multigrid on the same levels, on the GPU's own omegas and
    diagonals (as test_a_gpu_configs.test_vcycle_re3900_r0_r2)."""
    import torch
    import glsamd
    from mg_ref import OracleGMG
    d = deck(RE3900)
    meshes = [ShuffledMesh(d.mesh(r), seed=20 + r) for r in range(2)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=10)
    assert all(op.brick_shape != (0, 0, 0) for op in ops)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=10)
    for l in range(2):
        omega, lam = mg.relaxation(l)
        assert abs(lam - ref.estimate(l)) < 1e-3 * lam
    ref.set_omega([mg.relaxation(l)[0] for l in range(2)])
    for l in range(2):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        ref.invdiag[l] = dl.double().cpu().numpy()
    b = gi.rnd(5, meshes[1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    assert rel_err(dst.cpu().numpy(), ref.vcycle(b)) < 5e-4
