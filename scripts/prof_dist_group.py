#!/usr/bin/env python3
"""Rehearsal of the partitioned vmult's phase order on one GPU: an in-process
group of WORLD partitions of the Re3900 r2 mesh (gls_dist_vmult_group: the
phases of gls_dist_vmult with device copies in place of RCCL), 5 vmults.
Run under rocprofv3 --kernel-trace --memory-copy-trace; summarise with
scripts/dist_timeline.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))

import torch  # noqa: E402

import glsdist  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
mesh = d.mesh(2)
vel, p, slip = d.boundary_descriptor()
cmask = mesh.constraint_mask(vel, p, slip)
params, w = d.operator_parameters(2.5e-4)
u = gi.linearization_point(mesh.n_nodes, mesh.dim, d.u_max)
g = glsdist.LocalGroup(mesh, cmask, world, engine="gpu", native=True)
g.setup(params, u, gi.history(u, params["order"]), w)
srcs = g.scatter(gi.src_vector(mesh.n_dofs))
dsts = [r.new_vector() for r in g.ranks]
for _ in range(5):
    g.vmult(dsts, srcs)
torch.cuda.synchronize()
print("interior/total bricks per member:", [m.interior_bricks() for m in g.native])
