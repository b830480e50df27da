"""The sphere deck (input_sphere_amg.json): the gmsh 4.1
reader (glsmesh.read_msh, GridIn::read_msh of simulation.cc:858-872), the
unstructured coarse-mesh refinement and its boundary descriptor
(simulation.cc:876-893), checked against SURVEY §8d's counts; the oracle
(TEST INFRASTRUCTURE) against the KAT-1 partition of unity on the unstructured,
all-general-geometry mesh; GPU parity of vmult / residual on it.

Parity unpinned beyond the counts: the reference cannot be built here (no
deal.II), and the SphericalManifold of simulation.cc:868 is attached to a
manifold id no object carries, so refinement is flat."""
import os

import numpy as np
import pytest

import glsmesh as gm
from helpers import deck, deck_case, rel_err

SPHERE = "input_sphere_amg.json"
REF_MSH = "/root/reference/mesh/sphere.msh"


def test_coarse_arrays():
    with np.load(gm.SPHERE_COARSE) as z:
        assert z["vertices"].shape == (1337, 3) and z["cells"].shape == (1024, 8)
        assert sorted(set(z["bids"].tolist())) == [0, 1, 2, 3]
        # every coarse cell right-handed after read_msh's reordering
        p = z["vertices"][z["cells"]]
        jac = np.einsum("ci,ci->c", np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]),
                        p[:, 4] - p[:, 0])
        assert np.all(jac > 0)


@pytest.mark.skipif(not os.path.exists(REF_MSH), reason="reference checkout absent")
def test_reader_matches_converted_arrays():
    c = gm.read_msh(REF_MSH)
    with np.load(gm.SPHERE_COARSE) as z:
        for k in ("vertices", "cells", "bfaces", "bids"):
            assert np.array_equal(c[k], z[k]), k


@pytest.mark.parametrize("n_ref,cells,dofs", [(0, 1024, 37568), (1, 8192, 280952),
                                              (3, 524288, 17073608)])
def test_counts(n_ref, cells, dofs):
    m = deck(SPHERE).mesh(n_ref)
    assert (m.n_cells, m.n_dofs) == (cells, dofs)


def test_boundary_descriptor():
    d = deck(SPHERE)
    m = d.mesh(1)
    vel, p, slip = d.boundary_descriptor()
    cm = m.constraint_mask(vel, p, slip)
    nb = m.node_boundary
    sphere_nodes = (nb & 1) != 0
    assert np.all(cm[sphere_nodes] & 7 == 7)          # no-slip sphere (id 0)
    assert np.all(cm[(nb & 2) != 0] & 7 == 7)         # inflow (id 1)
    out = ((nb & 8) != 0) & ((nb & 7) == 0)
    assert np.all(cm[out] == 8)                       # outflow pressure (id 3)
    walls = (nb == 4)
    # slip walls y = +-5 / z = +-5: exactly the normal component
    y = np.abs(np.abs(m.coords[:, 1]) - 5) < 1e-12
    z = np.abs(np.abs(m.coords[:, 2]) - 5) < 1e-12
    assert np.all(cm[walls & y & ~z] == 2) and np.all(cm[walls & z & ~y] == 4)
    assert np.all(cm[walls & y & z] == 6)
    g = d.constraint_values(m)
    assert np.all(g[np.nonzero((nb & 2) != 0)[0] * 4] == 1.0)


def test_oracle_partition_of_unity():
    """KAT-1: constant velocity, zero pressure, constant linearization point
    (no constraints, order 0): sum of velocity rows = 0 for w0 = 0 and the
    pressure rows sum to 0 — the mass term is absent for "none"."""
    import oracle as orc
    case = deck_case(SPHERE, 0)
    m = case.mesh
    cm = np.zeros(m.n_nodes, dtype=np.uint8)
    om = orc.OracleMesh(m, cm)
    prm = dict(case.params)
    prm["w0"] = 1.0
    o = orc.Oracle(om, **prm)
    u = np.zeros(m.n_dofs)
    u[0::4], u[1::4], u[2::4] = 1.0, 0.5, -0.25
    o.set_linearization_point(u)
    dst = o.vmult(u).reshape(-1, 4)
    meas, _ = m.cell_measure()
    # sum_i dst_i^(d) = w0 c_d |Omega| with the Q2 geometry's volume
    vol = dst[:, 0].sum() / 1.0
    assert abs(dst[:, 1].sum() - 0.5 * vol) < 1e-9 * abs(vol)
    assert abs(dst[:, 2].sum() + 0.25 * vol) < 1e-9 * abs(vol)
    assert abs(dst[:, 3].sum()) < 1e-9 * abs(vol)
    assert abs(vol - meas.sum()) < 0.05 * meas.sum()   # box minus ball


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_gpu_vmult_residual_sphere(prec):
    import torch
    case = deck_case(SPHERE, 1)
    o = case.oracle()
    op = case.gpu(prec)
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.u_star))
    torch.cuda.synchronize()
    tol = 1e-12 if prec == "f64" else 1e-5
    assert rel_err(dst.double().cpu().numpy(), o.vmult(case.src)) < tol
    assert rel_err(res.double().cpu().numpy(), o.evaluate_residual(case.u_star)) < tol
