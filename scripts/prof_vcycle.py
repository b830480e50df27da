#!/usr/bin/env python3
"""20 FP32 V-cycles on the Re3900 r0..r2 hierarchy (for rocprofv3 --stats:
where the preconditioner's time goes)."""
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
# argv[1]: coarse solver (10 relaxation sweeps by default; -1 = the deck's
# direct solver, the dense free-dof inverse GEMV)
coarse = int(sys.argv[1]) if len(sys.argv) > 1 else 10
mg, ops = glsamd.build_gmg(meshes, cm, params, u, gi.history(u, 2), w, precision="f32",
                           coarse_n_iterations=coarse)
b = ops[-1]._dev(gi.src_vector(meshes[-1].n_dofs)).double()
x = torch.empty_like(b)
for _ in range(3):
    mg.vcycle(x, b)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    mg.vcycle(x, b)
torch.cuda.synchronize()
print(f"vcycle wall {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms")
