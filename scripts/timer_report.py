#!/usr/bin/env python3
"""The library's timer sections (gls_timer_*, the reference's MyTimerOutput
sections) over one Re3900 r2 setup + GMRES(28) solves: operator setup, the
r0..r2 FP32 multigrid setup (deck's direct coarse solve), three GMRES(28)
cycles (tolerance 0) with the FP64 operator -- the TimerOutput-style table
print_wall_time_statistics would print for the same work (main.cc:992).
Timing adds two events per section; the section times include them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import torch  # noqa: E402

import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

glsamd.timer_enable(True)
d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
meshes = [d.mesh(r) for r in range(3)]
vel, p, slip = d.boundary_descriptor()
cm = [m.constraint_mask(vel, p, slip) for m in meshes]
params, w = d.operator_parameters(2.5e-4)
u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
hist = gi.history(u, params["order"])
A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
A.set_parameters(**params)
A.set_linearization_point(u)
A.set_previous_solution(hist, w)
mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                           coarse_n_iterations=-1)
b = A._dev(gi.src_vector(meshes[-1].n_dofs))
x = A.initialize_dof_vector()
solver = glsamd.LinearSolverGMRES(A, mg, n_max_iterations=28, relative_tolerance=1e-30,
                                  absolute_tolerance=0.0)
for rep in range(3):
    x.zero_()
    try:
        solver.solve(x, b)
    except glsamd.GlsError:
        pass
torch.cuda.synchronize()
print(glsamd.timer_report())
