#!/usr/bin/env python3
"""The resident sweeps' failure mode, forced: with a build whose slot waits
give up at once (GLS_SWEEP_SPIN_MAX=0, lib/var/spin0.so through GLS_AMD_LIB)
hand-offs time out, gls_op_sweep_stats counts them and the V-cycle result
is NaN (the poisoned iterate), not a silently wrong smoothing."""
import os
import sys

import numpy as np

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
mg, ops = glsamd.build_gmg(meshes, cm, params, u, gi.history(u, 2), w, precision="f32",
                           coarse_n_iterations=10)
b = ops[-1]._dev(gi.src_vector(meshes[-1].n_dofs)).double()
x = torch.zeros_like(b)
mg.vcycle(x, b)
torch.cuda.synchronize()
stats = [op.sweep_stats() for op in ops]
n_nan = int(torch.isnan(x).sum())
print(f"resident launches / timeouts per level {stats}; NaN entries in the V-cycle result {n_nan}"
      f" of {x.numel()}")
sys.exit(0 if (sum(s[1] for s in stats) == 0 and n_nan == 0) or
         (sum(s[1] for s in stats) > 0 and n_nan > 0) else 1)
