#!/usr/bin/env python3
"""A/B of the two-layer FP32 bricks (GLS_TWO_LAYER, read at operator
creation): FP32 vmult back to back on the sphere r3 and Re3900 r3 meshes, and
the Turek-3D r0..r3 multigrid companion; alternating, twice."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))

import torch  # noqa: E402

import bench  # noqa: E402
import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402


def vmult_us(deck, n_ref, reps=50):
    d = gm.read_deck(os.path.join(gm.DECK_DIR, deck))
    params, w = d.operator_parameters(2.5e-4)
    m = d.mesh(n_ref)
    cm = m.constraint_mask(*d.boundary_descriptor())
    u = gi.linearization_point(m.n_nodes, m.dim, d.u_max)
    op = glsamd.NavierStokesOperator(m, cm, "f32")
    op.set_parameters(**params)
    op.set_linearization_point(u)
    if params["order"] > 0:
        op.set_previous_solution(gi.history(u, params["order"]), w)
    src = op._dev(gi.src_vector(m.n_dofs))
    dst = op.initialize_dof_vector()
    for _ in range(5):
        op.vmult(dst, src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        op.vmult(dst, src)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3, list(op.brick_shape)


res = {}
for rep in range(2):
    for v in ("0", "1"):
        os.environ["GLS_TWO_LAYER"] = v
        r = {"sphere_r3": vmult_us("input_sphere_amg.json", 3),
             "re3900_r3": vmult_us("input_hoffmann_3D_Re3900.json", 3)}
        t = bench.turek3d_mg_companion()
        r["turek3d"] = {k: t[next(iter(t))][k] for k in ("vcycle_ms", "gmres_iteration_ms")}
        res.setdefault(v, []).append(r)
        print(v, r, flush=True)
print(json.dumps(res))
