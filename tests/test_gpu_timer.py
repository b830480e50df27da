"""Timer sections (gls_timer_*, the reference's MyTimerOutput / MyScope
sections, timer.h:194-413): with timing on, the operator, multigrid and GMRES
entry points and the V-cycle phases are tallied under the reference's
section names (operator_ns.cc:200-761, multigrid.cc:207-450, 550-583,
solver_l.cc:49) with host and GPU times; off, nothing is tallied."""
import pytest

import glsinputs as gi
from helpers import deck

pytestmark = pytest.mark.gpu


def test_timer_sections():
    import torch
    import glsamd
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(2)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    was = glsamd.timer_enable(True)
    try:
        glsamd.timer_reset()
        A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
        A.set_parameters(**params)
        A.set_linearization_point(u)
        A.set_previous_solution(hist, w)
        mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                                 coarse_n_iterations=10)
        b = A._dev(gi.rnd(3, meshes[-1].n_dofs))
        x = A.initialize_dof_vector()
        for _ in range(3):
            A.vmult(x, b)
        for _ in range(2):
            mg.vcycle(x, b)
        solver = glsamd.LinearSolverGMRES(A, mg, n_max_iterations=5, relative_tolerance=1e-30,
                                          absolute_tolerance=0.0)
        x.zero_()
        try:
            solver.solve(x, b)
        except glsamd.GlsError:
            pass  # 5 iterations at tolerance 0
        n_it = solver.last["n_iterations"]
        torch.cuda.synchronize()
        t = glsamd.timer_sections()
        print(glsamd.timer_report())
        # the operator's own calls and one per GMRES iteration (+ the initial residual)
        assert t["ns::vmult"]["calls"] >= 3 + n_it
        assert t["ns::vmult"]["gpu_ms"] > 0
        assert t["ns::set_linearization_point"]["calls"] >= 1
        assert t["ns::set_previous_solution"]["calls"] >= 1
        assert t["gmg::initialize"]["calls"] == 1
        assert t["gmg::initialize::smoother::init0"]["calls"] == 2      # both levels
        assert t["gmg::initialize::smoother::init1"]["calls"] >= 1
        # two direct cycles, one per GMRES iteration (+ one for the update
        # when GMRES keeps no preconditioned directions)
        n_vc = t["gmg::vmult"]["calls"]
        assert 2 + n_it <= n_vc <= 3 + n_it
        assert t["gmres::solve"]["calls"] == 1
        for ph in ("0_pre_smoother_step", "1_residual_step", "2_restriction",
                   "3_prolongation", "5_post_smoother_step"):
            assert t[f"gmg::vmult::level_1::{ph}"]["calls"] == n_vc
        assert t["gmg::vmult::level_0"]["calls"] == n_vc
        # the V-cycle phases are disjoint stretches of the cycle's stream
        phases = sum(v["gpu_ms"] for k, v in t.items() if k.startswith("gmg::vmult::level_"))
        assert 0.5 * t["gmg::vmult"]["gpu_ms"] < phases <= 1.02 * t["gmg::vmult"]["gpu_ms"]
        assert t["gmres::solve"]["gpu_ms"] >= t["gmg::vmult"]["gpu_ms"] * n_it / n_vc * 0.9
        # off: nothing more is tallied
        glsamd.timer_enable(False)
        A.vmult(x, b)
        torch.cuda.synchronize()
        assert glsamd.timer_sections()["ns::vmult"]["calls"] == t["ns::vmult"]["calls"]
    finally:
        glsamd.timer_enable(was)
        glsamd.timer_reset()
