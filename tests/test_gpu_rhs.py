"""evaluate_residual / evaluate_rhs with the inhomogeneous constraints
distributed (operator_ns.cc:622-682: tmp = src;
constraints_inhomogeneous.distribute(tmp); residual cell loop; set_zero;
*= -1) against the oracle's residual cell loop (TEST INFRASTRUCTURE) on
the distributed vector.  The distribute step is restated here in numpy:
constrained components take the inflow values of
glsmesh.Deck.constraint_values (zero on the homogeneous rows).
FP64 relative l2 1e-12, FP32 1e-5 (as test_gpu_parity)."""
import numpy as np
import pytest

from helpers import deck_case, deck, rel_err

pytestmark = pytest.mark.gpu
TOL = {"f64": 1e-12, "f32": 1e-5}


def _np(t):
    return t.double().cpu().numpy()


def distribute(x, cmask, g):
    """AffineConstraints::distribute for Dirichlet-type constraints."""
    nc = x.size // cmask.size
    y = np.array(x, dtype=np.float64, copy=True)
    con = ((cmask[:, None] >> np.arange(nc)[None, :]) & 1).astype(bool).ravel()
    y[con] = g[con]
    return y


CASES = [("input_hoffmann_3D_Re3900.json", 1, 0.0), ("input_turek_2D_Re100.json", 2, 0.02),
         ("input_turek_2D_Re20_stat.json", 1, 0.0)]


@pytest.mark.parametrize("name,n_ref,t", CASES)
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_residual_and_rhs_distributed(name, n_ref, t, prec):
    import torch
    case = deck_case(name, n_ref)
    g = deck(name).constraint_values(case.mesh, t)
    assert np.any(g != 0)
    o = case.oracle()
    op = case.gpu(prec)
    op.set_constraint_values(g)
    res = op.initialize_dof_vector()
    op.evaluate_residual(res, op._dev(case.u_star))
    rhs = op.initialize_dof_vector()
    rhs.fill_(3.0)  # overwritten
    op.evaluate_rhs(rhs)
    torch.cuda.synchronize()
    ref_res = o.evaluate_residual(distribute(case.u_star, case.cmask, g))
    ref_rhs = o.evaluate_residual(distribute(np.zeros(case.n_dofs), case.cmask, g))
    assert np.linalg.norm(ref_rhs) > 0
    assert rel_err(_np(res), ref_res) < TOL[prec]
    assert rel_err(_np(rhs), ref_rhs) < TOL[prec]


def test_distribute_semantics():
    """No values set = all constrained values zero; clearing restores it;
    distributed == plain on an already distributed vector."""
    import torch
    case = deck_case("input_hoffmann_3D_Re3900.json", 1)
    g = deck("input_hoffmann_3D_Re3900.json").constraint_values(case.mesh)
    o = case.oracle()
    op = case.gpu("f64")
    res0 = op.initialize_dof_vector()
    op.evaluate_residual(res0, op._dev(case.src))
    rhs0 = op.initialize_dof_vector()
    op.evaluate_rhs(rhs0)
    torch.cuda.synchronize()
    assert rel_err(_np(res0), o.evaluate_residual(distribute(case.src, case.cmask,
                                                             np.zeros(case.n_dofs)))) < 1e-12
    # zero vector, zero constraints: only the BDF history term u_time_derivative_old
    # (operator_ns.cc:997-998) remains
    assert rel_err(_np(rhs0), o.evaluate_residual(np.zeros(case.n_dofs))) < 1e-12
    op.set_constraint_values(g)
    xd = op._dev(distribute(case.src, case.cmask, g))
    a, b = op.initialize_dof_vector(), op.initialize_dof_vector()
    op.evaluate_residual(a, op._dev(case.src))
    op.evaluate_residual_plain(b, xd)
    op.set_constraint_values(None)
    c = op.initialize_dof_vector()
    op.evaluate_residual(c, op._dev(case.src))
    torch.cuda.synchronize()
    # same arithmetic; the LDS-atomic accumulation order varies run to run
    assert rel_err(_np(a), _np(b)) < 1e-14
    assert rel_err(_np(c), _np(res0)) < 1e-14
