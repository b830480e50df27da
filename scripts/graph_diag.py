"""Diagnostic: V-cycle replayed from the captured graph vs launched kernel by
kernel, repeated calls with different inputs (Re3900 r0..r1, FP32)."""
import os, sys
sys.path[:0] = ['dealii-ns-gls_amd/python', 'oracle', 'tests']
import numpy as np, torch
import glsamd, glsinputs as gi
from helpers import deck
d = deck("input_hoffmann_3D_Re3900.json")
meshes = [d.mesh(r) for r in range(2)]
vel, p, slip = d.boundary_descriptor()
cm = [m.constraint_mask(vel, p, slip) for m in meshes]
params, w = d.operator_parameters(2.5e-4)
u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
hist = gi.history(u, params["order"])
n = meshes[-1].n_dofs
for mode in ("1", "2", "3"):
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32", coarse_n_iterations=int(sys.argv[1]) if len(sys.argv) > 1 else 10)
    out = []
    for it in range(3):
        b = torch.from_numpy(gi.rnd(20 + it, n)).cuda()
        os.environ["GLS_MG_GRAPH"] = "0"
        r = torch.zeros_like(b); mg.vcycle(r, b)
        os.environ["GLS_MG_GRAPH"] = mode
        g = torch.zeros_like(b); mg.vcycle(g, b)
        torch.cuda.synchronize()
        out.append(f"{float((g - r).norm() / r.norm()):.2e}")
    print("mode", mode, out, flush=True)
