"""Nonlinear solvers and their wiring: the host-side
mirror of solver_nl.{h,cc} (NonLinearSolverLinearized / Newton / Picard) and
of the Newton lambdas of main.cc:805-864, over the device-resident operator,
GMRES and multigrid of libglsamd.so.

The nonlinear loops are control logic (a handful of scalar decisions per
iteration, as in the reference); every vector they touch stays in HBM and
every operation on them is a library call (vmult / residual / GMRES /
V-cycle) or a torch elementwise op.  The callbacks have the reference's
names and argument order, so a driver that sets them up like main.cc does
works unchanged.
"""
from __future__ import annotations

import numpy as np

import glsamd


class NonLinearSolverBase:
    """solver_nl.h: the std::function hooks the driver fills in."""

    def __init__(self):
        self.setup_jacobian = None        # (solution)
        self.setup_preconditioner = None  # (solution)
        self.evaluate_rhs = None          # (dst)
        self.evaluate_residual = None     # (dst, src)
        self.solve_with_jacobian = None   # (dst, src)
        self.postprocess = None           # (solution)
        self.history = []                 # residual l2 norms per step (the "[N] step" log)


class NonLinearSolverLinearized(NonLinearSolverBase):
    """solver_nl.cc:4-24: one linear solve around the current solution."""

    def solve(self, solution):
        import torch
        self.setup_jacobian(solution)
        rhs = torch.zeros_like(solution)
        self.evaluate_rhs(rhs)
        self.setup_preconditioner(solution)
        self.solve_with_jacobian(solution, rhs)
        return 1


class NonLinearSolverNewton(NonLinearSolverBase):
    """solver_nl.cc:26-89: Newton on the residual; the preconditioner is set
    up at the first step only when inexact_newton.  Tolerance 1e-7 and at
    most 30 steps (solver_nl.cc:29-30); exceeding them raises, as the
    reference's AssertThrow."""

    def __init__(self, inexact_newton=True, newton_tolerance=1.0e-7, newton_max_iteration=30):
        super().__init__()
        self.inexact_newton = inexact_newton
        self.newton_tolerance = newton_tolerance
        self.newton_max_iteration = newton_max_iteration

    def solve(self, solution):
        with glsamd.timer_scope("newton::solve"):  # solver_nl.cc:38
            return self._solve(solution)

    def _solve(self, solution):
        import torch
        rhs = torch.zeros_like(solution)
        inc = torch.zeros_like(solution)
        self.setup_jacobian(solution)
        self.evaluate_residual(rhs, solution)
        l2 = float(rhs.norm())
        self.history = [l2]
        it = 0
        while l2 > self.newton_tolerance:
            inc.zero_()
            if it == 0 or not self.inexact_newton:
                self.setup_preconditioner(solution)
            self.solve_with_jacobian(inc, rhs)
            solution.add_(inc)
            if self.postprocess is not None:
                self.postprocess(solution)
            self.setup_jacobian(solution)
            self.evaluate_residual(rhs, solution)
            l2 = float(rhs.norm())
            it += 1
            self.history.append(l2)
            if it > self.newton_max_iteration:
                raise RuntimeError("Newton iteration did not converge. Final residual_0 is "
                                   f"{l2}.")
        return it


class NonLinearSolverPicard(NonLinearSolverBase):
    """solver_nl.cc:91-140: fixed-point iteration on the linearized operator,
    converged when the update's l2 norm drops below 1e-7."""

    def __init__(self, picard_tolerance=1.0e-7, picard_max_iteration=30):
        super().__init__()
        self.picard_tolerance = picard_tolerance
        self.picard_max_iteration = picard_max_iteration

    def solve(self, solution):
        import torch
        rhs = torch.zeros_like(solution)
        l2, it = 1e10, 0
        self.history = []
        while l2 > self.picard_tolerance:
            tmp = solution.clone()
            self.setup_jacobian(solution)
            self.evaluate_rhs(rhs)
            self.setup_preconditioner(solution)
            self.solve_with_jacobian(solution, rhs)
            l2 = float((tmp - solution).norm())
            it += 1
            self.history.append(l2)
            if it > self.picard_max_iteration:
                raise RuntimeError("Picard iteration did not converge. Final residual_0 is "
                                   f"{l2}.")
        return it


class GMGPreconditioner:
    """PreconditionerGMG with the main.cc:815-839 setup_preconditioner step:
    interpolate_to_mg of the current solution, set_linearization_point on
    every level operator, then PreconditionerGMG::initialize (inverse
    diagonals + power-iteration relaxation factors).  Histories of the
    levels are interpolated once, at construction (main.cc:772-803)."""

    def __init__(self, meshes, cmasks, params, solution, history=None, weights=None,
                 precision="f32", **mg_kwargs):
        self.mg, self.ops = glsamd.build_gmg(meshes, cmasks, params, solution, history,
                                             weights, precision=precision, **mg_kwargs)
        self.h = self.mg.h

    def initialize(self, solution):
        import torch
        vecs = [solution.to(self.ops[-1].dtype)]
        for l in range(len(self.ops) - 1, 0, -1):
            v = self.ops[l - 1].initialize_dof_vector()
            self.mg.interpolate(l, v, vecs[0])
            vecs.insert(0, v)
        for op, v in zip(self.ops, vecs):
            op.set_linearization_point(v)
        torch.cuda.synchronize()
        self.mg.setup()

    def vmult(self, dst, src):
        return self.mg.vcycle(dst, src)


def wire_newton(solver, op, cmask, linear_solver, preconditioner=None):
    """main.cc:805-864: setup_jacobian = set_linearization_point on the fine
    operator; setup_preconditioner = GMG initialize at the solution;
    evaluate_rhs / evaluate_residual = the operator's; solve_with_jacobian =
    set_zero(src) on constrained rows, GMRES, distribute(dst) (homogeneous:
    constrained increments 0)."""
    import torch
    nc = op.dim + 1
    cm = np.asarray(cmask, dtype=np.uint8)
    con = ((cm[:, None] >> np.arange(nc)[None, :]) & 1).astype(bool).ravel()
    con_t = torch.from_numpy(con).to("cuda")

    def setup_jacobian(src):
        op.set_linearization_point(src)

    def setup_preconditioner(solution):
        if preconditioner is not None:
            preconditioner.initialize(solution)
        linear_solver.initialize()

    def evaluate_rhs(dst):
        op.evaluate_rhs(dst)

    def evaluate_residual(dst, src):
        op.evaluate_residual(dst, src)

    def solve_with_jacobian(dst, src):
        src.masked_fill_(con_t, 0.0)
        linear_solver.solve(dst, src)
        dst.masked_fill_(con_t, 0.0)

    solver.setup_jacobian = setup_jacobian
    solver.setup_preconditioner = setup_preconditioner
    solver.evaluate_rhs = evaluate_rhs
    solver.evaluate_residual = evaluate_residual
    solver.solve_with_jacobian = solve_with_jacobian
    return solver
