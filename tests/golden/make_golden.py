#!/usr/bin/env python3
"""Generate the golden fixtures of tests/test_golden.py.

The reference (peterrum/dealii-ns-gls) needs deal.II + p4est + Trilinos,
none of which exists in this image, and ships no golden data of its own
(SURVEY §8c): these fixtures are outputs of OUR CPU restatement
(oracle/gls_oracle.c), pinned by the known-answer tests of
tests/test_oracle_kat.py — parity against the reference binary is unpinned.
They freeze the oracle's and the mesh generator's behaviour so that (a) the
CPU suite detects any drift of either, and (b) the GPU suite checks the HIP
path against stored numbers without running the oracle.

Inputs are the deterministic §8d synthetic vectors (glsinputs.py), so a
fixture stores only the outputs plus a digest of the mesh.

  python tests/golden/make_golden.py        (writes tests/golden/*.npz)
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "dealii-ns-gls_amd", "python"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402
import oracle as orc  # noqa: E402

# (fixture name, deck, refinements, overrides of the deck's operator flags)
CASES = [
    ("turek2d_re20_stat_r1", "input_turek_2D_Re20_stat.json", 1, {}),
    ("turek2d_re100_r1", "input_turek_2D_Re100.json", 1, {}),
    ("turek3d_re100_r0", "input_turek_3D_Re100.json", 0, {}),
    ("hoffmann3d_re3900_r0", "input_hoffmann_3D_Re3900.json", 0, {}),
    ("hoffmann3d_re3900_r0_fixed_cw", "input_hoffmann_3D_Re3900.json", 0,
     {"increment_form": False, "cell_wise_stabilization": True}),
]
DT = 2.5e-4


def mesh_digest(m):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(m.cell_nodes, dtype=np.uint32).tobytes())
    h.update(np.round(np.ascontiguousarray(m.coords), 12).tobytes())
    return h.hexdigest()


def case_inputs(deck_name, n_ref, overrides):
    d = gm.read_deck(os.path.join(gm.DECK_DIR, deck_name))
    m = d.mesh(n_ref)
    vel, p, slip = d.boundary_descriptor()
    cmask = m.constraint_mask(vel, p, slip)
    params, w = d.operator_parameters(DT)
    params.update(overrides)
    src = gi.src_vector(m.n_dofs)
    u = gi.linearization_point(m.n_nodes, m.dim, d.u_max)
    hist = gi.history(u, params["order"])
    return m, cmask, params, w, src, u, hist


def oracle_outputs(m, cmask, params, w, src, u, hist):
    om = orc.OracleMesh(m, cmask)
    o = orc.Oracle(om, **params)
    o.set_linearization_point(u)
    if params["order"] > 0:
        o.set_previous_solution(hist, w)
    return dict(vmult=o.vmult(src), residual=o.evaluate_residual(src),
                inverse_diagonal=o.inverse_diagonal())


def main():
    for name, deck, n_ref, ov in CASES:
        m, cmask, params, w, src, u, hist = case_inputs(deck, n_ref, ov)
        out = oracle_outputs(m, cmask, params, w, src, u, hist)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), n_cells=m.n_cells,
                            n_nodes=m.n_nodes, mesh_sha256=mesh_digest(m),
                            n_constrained=int(np.count_nonzero(cmask)), **out)
        print(name, m.n_cells, m.n_dofs)


if __name__ == "__main__":
    main()
