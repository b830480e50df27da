#!/usr/bin/env python3
"""Threaded in-process group vmults (one host thread + stream pair per
member: gls_dist_vmult's production schedule, device copies as transport)
for a kernel / memory-copy trace:
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- \\
      python3 scripts/prof_dist_threaded.py [world] [nref] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))


def main():
    import time
    import glsdist
    import glsinputs as gi
    import glsmesh as gm
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nref = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
    m = d.mesh(nref)
    cm = m.constraint_mask(*d.boundary_descriptor())
    prm, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(m.n_nodes, m.dim, d.u_max)
    g = glsdist.LocalGroup(m, cm, world, engine="gpu", native=True)
    g.setup(prm, u, gi.history(u, prm["order"]), w)
    srcs = g.scatter(gi.src_vector(m.n_dofs))
    dsts = [r.new_vector() for r in g.ranks]
    g.vmult_threaded(dsts, srcs, reps=3)
    t0 = time.perf_counter()
    g.vmult_threaded(dsts, srcs, reps=reps)
    el = (time.perf_counter() - t0) / reps
    print(f"threaded world {world} r{nref}: {el * 1e6:.1f} us per vmult (wall, all members on "
          f"one GPU)", flush=True)


if __name__ == "__main__":
    main()
