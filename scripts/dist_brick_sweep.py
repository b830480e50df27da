#!/usr/bin/env python3
"""Rank-local vmult time of the Re3900 r2 operator as the multi-GPU bench
partitions it (glsdist.build_partitions, world = 1, 2, 4, 8; the largest
rank), for several brick shapes: does a smaller work unit pay once a rank's
bricks no longer fill the GPU?  Single GPU, no exchange (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import glsamd  # noqa: E402
import glsdist  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
mesh = d.mesh(2)
vel, p, slip = d.boundary_descriptor()
cm = mesh.constraint_mask(vel, p, slip)
params, w = d.operator_parameters(2.5e-4)
u = gi.linearization_point(mesh.n_nodes, 3, d.u_max)
hist = gi.history(u, params["order"])
for world in (1, 2, 4, 8):
    parts = glsdist.build_partitions(mesh, world)
    part = max(parts, key=lambda q: q.n_cells)
    lm = glsdist.LocalMesh(mesh, part)
    lcm = np.asarray(cm)[part.local_nodes]
    lu = u.reshape(-1, 4)[part.local_nodes].ravel()
    lh = [h.reshape(-1, 4)[part.local_nodes].ravel() for h in hist]
    src = gi.src_vector(mesh.n_dofs).reshape(-1, 4)[part.local_nodes].ravel()
    line = []
    for shape in ((4, 4, 1), (4, 2, 1), (4, 1, 1)):
        op = glsamd.NavierStokesOperator(lm, lcm, "f64", n_owned_nodes=part.n_owned, brick=shape)
        op.set_parameters(**params)
        op.set_linearization_point(lu)
        op.set_previous_solution(lh, w)
        s = op._dev(src)
        dst = op.initialize_dof_vector()
        for _ in range(5):
            op.vmult(dst, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            op.vmult(dst, s)
        e1.record()
        torch.cuda.synchronize()
        line.append(f"{shape}: {e0.elapsed_time(e1) / 50 * 1e3:6.1f} us")
        del op
    print(f"world {world}: rank cells {part.n_cells}, " + ", ".join(line), flush=True)
