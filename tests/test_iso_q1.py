"""FE_Q_iso_Q1 coarsest multigrid level (main.cc:436-446, "gmg coarse grid
use fe q iso q1" of the sphere and Re20 decks): glsmesh.IsoQ1Mesh runs it as
the Q1 operator on the coarse cells' sub-cells (same support points, QGauss(2)
per sub-cell = QIterated(QGauss(2), k)), and the transfer to the next level
is the Q1 one (the iso-Q1 embedding).

CPU: structure (sub-cell corners are next-level nodes, measures add up) and
the oracle transfer's exactness on linear fields through the iso-Q1 level.
GPU: the V-cycle with an iso-Q1 coarse level against the oracle multigrid on
the same levels (the GPU's own omegas / diagonals, as test_gpu_mg.py)."""
import numpy as np
import pytest

import glsinputs as gi
import glsmesh as gm
import oracle as orc
from helpers import deck, rel_err

DECKS = [("input_sphere_amg.json", 1), ("input_turek_2D_Re20_stat.json", 2)]


@pytest.mark.parametrize("name,n_ref", DECKS)
def test_structure(name, n_ref):
    d = deck(name)
    assert d.use_fe_q_iso_q1
    m0, m1 = d.mesh(0), d.mesh(1)
    iso = gm.IsoQ1Mesh(m0)
    assert iso.degree == 1 and iso.n_nodes == m0.n_nodes
    assert iso.n_cells == m0.n_cells * m0.degree ** m0.dim
    ch = iso.child_lattice(m1)
    corners = [0, 2, 6, 8, 18, 20, 24, 26] if m0.dim == 3 else [0, 2, 6, 8]
    assert np.abs(np.asarray(m1.coords)[ch[:, corners]] -
                  np.asarray(m0.coords)[iso.cell_nodes]).max() < 1e-13
    meas, _ = iso.cell_measure()
    assert np.isclose(meas.sum(), m0.cell_measure()[0].sum())


@pytest.mark.parametrize("name,n_ref", DECKS)
def test_iso_transfer_linear_exact(name, n_ref):
    """Prolongation from the iso-Q1 level reproduces a linear field at the
    next level's nodes (multilinear geometry); interpolation back is the
    identity (KAT-6 style)."""
    d = deck(name)
    m0, m1 = d.mesh(0), d.mesh(1)
    iso = gm.IsoQ1Mesh(m0)
    dim, nc = m0.dim, m0.dim + 1
    om0 = orc.OracleMesh(iso, np.zeros(iso.n_nodes, np.uint8))
    om1 = orc.OracleMesh(m1, np.zeros(m1.n_nodes, np.uint8))
    child = iso.child_lattice(m1)
    a = np.array([[0.3, -1.2, 0.7][:dim], [1.1, 0.4, -0.5][:dim], [-0.2, 0.9, 0.6][:dim],
                  [0.5, 0.5, -1.0][:dim]])[:nc]
    f = lambda X: (X @ a.T + np.arange(nc)).ravel()  # noqa: E731
    uc = f(np.asarray(m0.coords))
    uf = np.zeros(m1.n_dofs)
    orc.prolongate_add(om0, om1, child, uf, uc)
    if d.simulation == "sphere":
        # multilinear cells: the reference-space embedding reproduces a
        # physically linear field (on the MappingQ2-curved cylinder cells it
        # reproduces the nodal interpolant in reference coordinates instead)
        assert np.abs(uf - f(np.asarray(m1.coords))).max() < 1e-12
    back = np.zeros(m0.n_dofs)
    orc.interpolate(om0, om1, child, back, uf)
    assert np.abs(back - uc).max() < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_ref,coarse", [("input_sphere_amg.json", 1, 10),
                                               ("input_turek_2D_Re20_stat.json", 2, -1)])
def test_gpu_vcycle_iso_q1(name, n_ref, coarse):
    import torch
    import glsamd
    from mg_ref import OracleGMG
    d = deck(name)
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=coarse, coarse_iso_q1=True)
    assert ops[0].degree == 1 and ops[0].n_cells == meshes[0].n_cells * 2 ** meshes[0].dim
    ref = OracleGMG([gm.IsoQ1Mesh(meshes[0])] + meshes[1:], cm, params, u, hist, w,
                    coarse_iters=coarse)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        ref.invdiag[l] = dl.double().cpu().numpy()
    # the level-0 operator itself: FP32 iso-Q1 GPU vs FP64 oracle on the sub-cells
    x0 = gi.rnd(3, meshes[0].n_dofs)
    y0 = ops[0].initialize_dof_vector()
    ops[0].vmult(y0, ops[0]._dev(x0))
    torch.cuda.synchronize()
    assert rel_err(y0.double().cpu().numpy(), ref.ops[0].vmult(x0)) < 2e-5
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    assert rel_err(dst.cpu().numpy(), ref.vcycle(b)) < 5e-4
