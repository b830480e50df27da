#!/usr/bin/env python3
"""Back-to-back vmult time of one deck / refinement / precision (the
library and GLS_* switches from the environment; A/B drivers loop over
them):  python scripts/time_vmult.py input_sphere_amg.json 3 f64 [reps]
prints "<deck> r<n> <prec> <us per vmult> <DoF/s>"; an optional fifth
argument "bx,by,bz" forces the brick shape (cells consecutive in the
mesh order); a sixth argument "det" sets GLS_DETERMINISTIC."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))


def main():
    import torch
    import glsamd
    import glsinputs as gi
    import glsmesh as gm
    deck, nref, prec = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    d = gm.read_deck(os.path.join(gm.DECK_DIR, deck))
    m = d.mesh(nref)
    cm = m.constraint_mask(*d.boundary_descriptor())
    prm, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(m.n_nodes, m.dim, d.u_max)
    brick = (tuple(int(x) for x in sys.argv[5].split(","))
             if len(sys.argv) > 5 and sys.argv[5] != "-" else None)
    op = glsamd.NavierStokesOperator(m, cm, prec, brick=brick)
    if len(sys.argv) > 6 and sys.argv[6] == "det":
        prm = dict(prm, deterministic=True)
    op.set_parameters(**prm)
    op.set_linearization_point(u)
    if prm["order"] > 0:
        op.set_previous_solution(gi.history(u, prm["order"]), w)
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
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{deck} r{nref} {prec} {us:.2f} {m.n_dofs / (us * 1e-6):.4g} brick {op.brick_shape}",
          flush=True)


if __name__ == "__main__":
    main()
