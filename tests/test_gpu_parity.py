"""GPU parity: HIP operator (through the C-ABI) vs the CPU oracle on the same
mesh and §8d synthetic inputs.

Tolerances (stated per north_star): FP64 relative l2 <= 1e-12 (atomic
scatter reorders sums), FP32 relative l2 <= 2e-5."""
import numpy as np
import pytest

from helpers import DECKS, deck_case, rel_err

pytestmark = pytest.mark.gpu
TOL = {"f64": 1e-12, "f32": 2e-5}


def _to_np(t):
    return t.double().cpu().numpy()


@pytest.mark.parametrize("name", DECKS)
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_vmult_decks(name, prec):
    import torch
    n_ref = {"input_turek_2D_Re100.json": 2, "input_turek_3D_Re100.json": 0,
             "input_hoffmann_3D_Re3900.json": 1}.get(name, None)
    case = deck_case(name, n_ref)
    o = case.oracle()
    op = case.gpu(prec)
    ref = o.vmult(case.src)
    src = op._dev(case.src)
    dst = op.initialize_dof_vector()
    op.vmult(dst, src)
    torch.cuda.synchronize()
    assert rel_err(_to_np(dst), ref) < TOL[prec]


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("variant", ["fixed", "cellwise", "theta"])
def test_vmult_variants(prec, variant):
    import torch
    over = {}
    if variant == "fixed":
        over = dict(nonlinear_solver="Picard")
    elif variant == "cellwise":
        over = dict(cell_wise_stabilization=True)
    elif variant == "theta":
        over = dict(time_integration="theta", theta=0.5, consider_time_derivative=False,
                    nonlinear_solver="Picard")
    case = deck_case("input_turek_2D_Re20_stat.json", 1, **over)
    o = case.oracle()
    op = case.gpu(prec)
    ref = o.vmult(case.src)
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    res_ref = o.evaluate_residual(case.src)
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.src))
    torch.cuda.synchronize()
    assert rel_err(_to_np(dst), ref) < TOL[prec]
    assert rel_err(_to_np(res), res_ref) < TOL[prec]


@pytest.mark.parametrize("name", ["input_turek_2D_Re100.json", "input_hoffmann_3D_Re3900.json"])
def test_tables_producers(name):
    case = deck_case(name, 0)
    o = case.oracle()
    op = case.gpu("f64")
    t_ref, cw_ref = o.tables()
    t, cw = op.download_tables()
    assert rel_err(t, t_ref) < 1e-13
    assert rel_err(cw, cw_ref) < 1e-13


@pytest.mark.parametrize("name", ["input_turek_2D_Re20_stat.json", "input_hoffmann_3D_Re3900.json"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_inverse_diagonal(name, prec):
    import torch
    case = deck_case(name, 0)
    o = case.oracle()
    op = case.gpu(prec)
    ref = o.inverse_diagonal()
    d = op.initialize_dof_vector()
    op.compute_inverse_diagonal(d)
    torch.cuda.synchronize()
    assert rel_err(_to_np(d), ref) < TOL[prec] * 10


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_residual_3d(prec):
    import torch
    case = deck_case("input_hoffmann_3D_Re3900.json", 0)
    o = case.oracle()
    op = case.gpu(prec)
    ref = o.evaluate_residual(case.u_star)
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.u_star))
    torch.cuda.synchronize()
    assert rel_err(_to_np(res), ref) < TOL[prec]


# The headline workload (Re3900 r2, BASELINE.json configs[3]): 4x4x1 bricks run
# in two rounds of 8 cells per workgroup and the persistent grid walks several
# bricks per workgroup, which the r0/r1 decks above (one round, one brick per
# workgroup) do not reach.  Smaller bricks change the round count and the
# shared-node structure; all must give the same operator.
@pytest.fixture(scope="module")
def re3900_r2():
    case = deck_case("input_hoffmann_3D_Re3900.json", 2)
    o = case.oracle()
    return case, o.vmult(case.src), o.evaluate_residual(case.u_star)


@pytest.mark.parametrize("brick", [None, (4, 2, 1), (4, 1, 1)])
def test_vmult_headline_r2(re3900_r2, brick):
    import torch
    case, ref, _ = re3900_r2
    op = case.gpu("f64", brick=brick)
    dst = op.initialize_dof_vector()
    src = op._dev(case.src)
    for _ in range(2):  # repeated applies overwrite dst completely
        op.vmult(dst, src)
    torch.cuda.synchronize()
    assert rel_err(_to_np(dst), ref) < TOL["f64"]


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_residual_headline_r2(re3900_r2, prec):
    import torch
    case, _, ref = re3900_r2
    op = case.gpu(prec)
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.u_star))
    torch.cuda.synchronize()
    assert rel_err(_to_np(res), ref) < TOL[prec]
