"""GPU parity of the weak outflow boundary-face terms (faces.hip) against the
oracle (tests/test_outflow_oracle.py pins the oracle's face terms by known
answers): vmult, residual (with the Nitsche target g = the inflow function at
the face points, simulation.cc:398), inverse diagonal and the system matrix,
on the cylinder decks with their outflow switched to "cut" / "nitsche"
(simulation.cc:270-278, 394-403: id 1 leaves the pressure free), brick and
per-cell kernels; and a GMRES + GMG solve whose level operators carry the
faces too (main.cc:510-527), checked by the oracle's true residual.

Tolerances as test_gpu_parity: FP64 relative l2 1e-12, FP32 2e-5."""
import numpy as np
import pytest

import glsmesh as gm
from helpers import deck, deck_case, rel_err

pytestmark = pytest.mark.gpu
TOL = {"f64": 1e-12, "f32": 2e-5}
CASES = [("input_turek_2D_Re20_stat.json", 1), ("input_turek_2D_Re100.json", 1),
         ("input_hoffmann_3D_Re3900.json", 1)]


def _np(t):
    return t.double().cpu().numpy()


def _case(name, n_ref, kind, u_back=0.0):
    case = deck_case(name, n_ref, outflow_bc=kind)
    cells, fno = gm.boundary_faces(case.mesh, 1)
    assert len(cells) > 0
    if u_back:
        # a linearization point with backflow through part of the outflow,
        # so that min(0, u* . n) is active on some faces
        nc = case.dim + 1
        x = case.mesh.coords
        scale = 1.0 + np.abs(case.u_star[0::nc]).max()
        case.u_star[0::nc] -= u_back * scale * (x[:, 1] > np.median(x[:, 1]))
    return case, (cells, fno, kind)


@pytest.mark.parametrize("name,n_ref", CASES)
@pytest.mark.parametrize("kind", ["cut", "nitsche"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_outflow_vmult_residual(name, n_ref, kind, prec):
    import torch
    case, of = _case(name, n_ref, kind, u_back=2.0 if kind == "cut" else 0.0)
    d = deck(name)
    o = case.oracle(outflow=of)
    op = case.gpu(prec, outflow=of)
    assert op.n_outflow_faces[0] == len(of[0])
    pts = op.outflow_face_points()
    assert rel_err(pts, o.outflow_face_points()) < 1e-14
    g = d.inflow_velocity(pts, 0.1, case.mesh.params["height"])
    o.set_outflow_target(g)
    op.set_outflow_target(g)
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.u_star))
    dg = op.initialize_dof_vector()
    op.compute_inverse_diagonal(dg)
    torch.cuda.synchronize()
    ref = o.vmult(case.src)
    # the face terms are a visible part of the operator
    assert rel_err(ref, case.oracle().vmult(case.src)) > 1e-6
    assert rel_err(_np(dst), ref) < TOL[prec]
    assert rel_err(_np(res), o.evaluate_residual(case.u_star)) < TOL[prec]
    # the assembled diagonal (1 / inverse): the backflow faces' negative
    # entries nearly cancel some cell diagonals, which FP32 inverts to a
    # large relative error in those few entries only
    assert rel_err(1 / _np(dg), 1 / o.inverse_diagonal()) < TOL[prec] * 10


@pytest.mark.parametrize("kind", ["cut", "nitsche"])
def test_outflow_per_cell_and_system_matrix(kind):
    import torch
    case, of = _case("input_hoffmann_3D_Re3900.json", 0, kind, u_back=2.0)
    o = case.oracle(outflow=of)
    op = case.gpu("f64", brick=(0, 0, 0), outflow=of)
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    torch.cuda.synchronize()
    ref = o.vmult(case.src)
    assert rel_err(_np(dst), ref) < TOL["f64"]
    A = case.gpu("f64", outflow=of).system_matrix()
    assert rel_err(A @ case.src, ref) < TOL["f64"]
    E = op.element_matrices()
    for c in np.unique(of[0])[:4]:
        assert rel_err(E[c], o.cell_matrix(int(c))) < TOL["f64"]


def test_outflow_gmres_gmg():
    """Nitsche outflow on every level: the FP32 V-cycle (unfused smoother,
    the face terms need the whole A x) preconditions GMRES on the r1 Newton
    system; the solution meets the tolerance in the oracle's operator."""
    import torch
    import glsamd
    import glsinputs as gi
    from helpers import Case
    name = "input_hoffmann_3D_Re3900.json"
    d = deck(name)
    d.outflow_bc = "nitsche"
    meshes = [d.mesh(r) for r in range(2)]
    vel, p, slip = d.boundary_descriptor()
    assert p == []
    cmasks = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32",
                               coarse_n_iterations=10, outflow=("nitsche", 1))
    assert all(op.n_outflow_faces[0] > 0 for op in ops)
    of = (*gm.boundary_faces(meshes[-1], 1), "nitsche")
    A = glsamd.NavierStokesOperator(meshes[-1], cmasks[-1], "f64", outflow=of)
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    b = gi.rnd(3, meshes[-1].n_dofs)
    solver = glsamd.LinearSolverGMRES(A, mg, n_max_iterations=400, relative_tolerance=1e-6)
    x = A.initialize_dof_vector()
    solver.solve(x, A._dev(b))
    torch.cuda.synchronize()
    st = solver.last
    cs = Case(meshes[-1], cmasks[-1], params, w, d.u_max)
    o = cs.oracle(outflow=of)
    true_res = np.linalg.norm(b - o.vmult(_np(x)))
    print("outflow gmres", st)
    assert st["converged"] == 1
    assert true_res <= 64 * st["tolerance"], (true_res, st)


def test_outflow_bad_face_rejected():
    """An invalid outflow face fails gls_op_create loudly (and frees what the
    create had built); a partitioned operator refuses faces."""
    import glsamd
    case, (cells, fno, kind) = _case("input_turek_2D_Re20_stat.json", 0, "nitsche")
    bad = fno.copy()
    bad[0] = 7
    with pytest.raises(glsamd.GlsError, match="outflow face"):
        case.gpu("f64", outflow=(cells, bad, kind))
    with pytest.raises(glsamd.GlsError, match="single domain"):
        glsamd.NavierStokesOperator(case.mesh, case.cmask, "f64",
                                    n_owned_nodes=case.mesh.n_nodes - 1,
                                    outflow=(cells, fno, kind))
