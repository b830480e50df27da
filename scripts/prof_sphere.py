#!/usr/bin/env python3
"""Kernel trace of the sphere deck's V-cycle (input_sphere_amg.json r3:
FE_Q_iso_Q1 coarse level, coarse GMRES to 1e-4 preconditioned by the AMG):
4 V-cycles after the setup; scripts/vtrace_summary.py attributes the
second-to-last one.  argv[1] = "relax10": 10 relaxation sweeps instead of
the AMG."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))

import torch  # noqa: E402

import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_sphere_amg.json"))
params, w = d.operator_parameters(2.5e-4)
meshes = [d.mesh(r) for r in range(d.n_refinements + 1)]
vel, p, slip = d.boundary_descriptor()
cm = [m.constraint_mask(vel, p, slip) for m in meshes]
u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
kw = (dict(coarse_n_iterations=10) if len(sys.argv) > 1 and sys.argv[1] == "relax10"
      else dict(coarse_amg=d.amg_parameters()))
mg, _ = glsamd.build_gmg(meshes, cm, params, u, gi.history(u, params["order"]), w,
                         precision="f32", coarse_iso_q1=True, coarse_iterate=True,
                         coarse_reltol=1e-4, coarse_maxiter=2000, **kw)
b = torch.from_numpy(gi.src_vector(meshes[-1].n_dofs)).cuda()
x = torch.zeros_like(b)
for _ in range(4):
    mg.vcycle(x, b)
torch.cuda.synchronize()
print("coarse GMRES iterations / converged:", mg.coarse_statistics())
