#!/usr/bin/env python3
"""Five GMRES(28) cycles (tolerance 0: 28 iterations each) on the Re3900 r2
FP64 operator with the r0..r2 FP32 multigrid (relaxation coarse solve), for
rocprofv3 --kernel-trace --stats: where a GMRES iteration's time goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import torch  # noqa: E402

import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
meshes = [d.mesh(r) for r in range(3)]
vel, p, slip = d.boundary_descriptor()
cm = [m.constraint_mask(vel, p, slip) for m in meshes]
params, w = d.operator_parameters(2.5e-4)
u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
hist = gi.history(u, params["order"])
mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                           coarse_n_iterations=10)
A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
A.set_parameters(**params)
A.set_linearization_point(u)
A.set_previous_solution(hist, w)
b = A._dev(gi.src_vector(meshes[-1].n_dofs))
x = A.initialize_dof_vector()
solver = glsamd.LinearSolverGMRES(A, mg, n_max_iterations=28, relative_tolerance=1e-30,
                                  absolute_tolerance=0.0)
for rep in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        solver.solve(x, b)
    except glsamd.GlsError:
        pass
    torch.cuda.synchronize()
    print(f"gmres {solver.last['n_iterations']} its, {(time.perf_counter() - t0) * 1e3:.2f} ms")
