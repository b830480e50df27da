"""One implicit time step's Newton solve on the GPU:
NonLinearSolverNewton (solver_nl.cc:26-89) wired as main.cc:805-864 —
fine FP64 operator, FP32 GMG preconditioner set up at the first step
(inexact Newton), device GMRES with the deck's relative tolerance — on the
Re3900 deck at r1 (BDF2, increment form).  The converged solution's residual
is recomputed by the oracle (TEST INFRASTRUCTURE) on the CPU, with the
inhomogeneous constraints distributed, and must meet the Newton tolerance;
the solution must satisfy the Dirichlet values exactly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_newton_time_step_re3900():
    import torch
    import glsamd
    import glsinputs as gi
    import glssolvers as gs
    from helpers import Case, deck
    from test_gpu_rhs import distribute
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(2)]
    vel, p, slip = d.boundary_descriptor()
    cmasks = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    fine = meshes[-1]
    g = d.constraint_values(fine, 0.0)
    u_old = gi.linearization_point(fine.n_nodes, fine.dim, d.u_max)
    hist = gi.history(u_old, params["order"])
    # the start value of the step: the old solution with this step's
    # Dirichlet values distributed (main.cc:893 / 943)
    u0 = distribute(u_old, cmasks[-1], g)
    op = glsamd.NavierStokesOperator(fine, cmasks[-1], "f64")
    op.set_parameters(**params)
    op.set_linearization_point(u0)
    op.set_previous_solution(hist, w)
    op.set_constraint_values(g)
    pre = gs.GMGPreconditioner(meshes, cmasks, params, u0, hist, w, precision="f32",
                               coarse_n_iterations=10)
    lin = glsamd.LinearSolverGMRES(op, pre, n_max_iterations=1000, relative_tolerance=1e-2)
    newton = gs.wire_newton(gs.NonLinearSolverNewton(inexact_newton=True, newton_tolerance=1e-7),
                            op, cmasks[-1], lin, pre)
    sol = op._dev(u0)
    n_it = newton.solve(sol)
    torch.cuda.synchronize()
    print("newton steps", n_it, "residuals", newton.history)
    assert 1 <= n_it <= 30
    assert newton.history[-1] <= 1e-7 < newton.history[0]
    x = sol.double().cpu().numpy()
    # Dirichlet values hold exactly (increments are zero on constrained rows)
    con = ((cmasks[-1][:, None] >> np.arange(4)[None, :]) & 1).astype(bool).ravel()
    assert np.array_equal(x[con], g[con])
    # the oracle's residual of the converged solution
    case = Case(fine, cmasks[-1], params, w, d.u_max)
    case.u_star = x
    case.hist = hist
    o = case.oracle()
    r = o.evaluate_residual(distribute(x, cmasks[-1], g))
    assert np.linalg.norm(r) <= 1e-6, np.linalg.norm(r)
