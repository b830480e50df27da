"""Diagnostic: the Newton test's solve (Re3900 r1) with the V-cycle graph on
and off: Newton residual history and GMRES iterations per step."""
import os, sys
sys.path[:0] = ['dealii-ns-gls_amd/python', 'oracle', 'tests']
import numpy as np, torch
import glsamd, glsinputs as gi, glssolvers as gs
from helpers import deck
from test_gpu_rhs import distribute
for env in [{"GLS_MG_GRAPH": "0"}, {}]:
    os.environ.pop("GLS_MG_GRAPH", None)
    os.environ.update(env)
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(2)]
    vel, p, slip = d.boundary_descriptor()
    cmasks = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    fine = meshes[-1]
    g = d.constraint_values(fine, 0.0)
    u_old = gi.linearization_point(fine.n_nodes, fine.dim, d.u_max)
    hist = gi.history(u_old, params["order"])
    u0 = distribute(u_old, cmasks[-1], g)
    op = glsamd.NavierStokesOperator(fine, cmasks[-1], "f64")
    op.set_parameters(**params)
    op.set_linearization_point(u0)
    op.set_previous_solution(hist, w)
    op.set_constraint_values(g)
    pre = gs.GMGPreconditioner(meshes, cmasks, params, u0, hist, w, precision="f32",
                               coarse_n_iterations=10)
    lin = glsamd.LinearSolverGMRES(op, pre, n_max_iterations=1000, relative_tolerance=1e-2)
    its = []
    orig = lin.solve
    def solve(dst, src):
        try:
            return orig(dst, src)
        finally:
            its.append(lin.last["n_iterations"])
    lin.solve = solve
    newton = gs.wire_newton(gs.NonLinearSolverNewton(inexact_newton=True, newton_tolerance=1e-7),
                            op, cmasks[-1], lin, pre)
    sol = op._dev(u0)
    try:
        n_it = newton.solve(sol)
        st = f"converged in {n_it}"
    except Exception as e:
        st = str(e)[:100]
    print(env, st, "gmres its", its, "hist", [f"{h:.2e}" for h in newton.history], flush=True)
