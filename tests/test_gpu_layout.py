"""The reference's vector layout through the C-ABI: vectors in HOST memory
(LinearAlgebra::distributed::Vector<Number>, config.h:9-10) and in a
caller (deal.II DoFHandler-like) numbering, via gls_op_set_vector_layout /
gls_mg_set_vector_layout.  Results must equal the default device /
node-major path permuted (the same kernels run on the same
node-major data, up to the LDS-atomic summation order) and the oracle (FP64 1e-12); get_max_u against the oracle
(operator_ns.cc:530-568)."""
import numpy as np
import pytest

import glsinputs as gi
from helpers import deck, deck_case, rel_err

pytestmark = pytest.mark.gpu


def _perm(n, seed=5):
    return np.random.default_rng(seed).permutation(n).astype(np.int64)


def test_operator_host_permuted():
    import torch
    case = deck_case("input_hoffmann_3D_Re3900.json", 1)
    o = case.oracle()
    ref = o.vmult(case.src)
    perm = _perm(case.n_dofs)           # caller dof i -> node-major dof perm[i]
    op = case.gpu("f64")
    op.set_vector_layout("host", perm)
    op.set_linearization_point(case.u_star[perm])
    op.set_previous_solution([h[perm] for h in case.hist], case.weights)
    dst = np.zeros(case.n_dofs)
    op.vmult(dst, np.ascontiguousarray(case.src[perm]))
    assert rel_err(dst, ref[perm]) < 1e-12
    res = np.zeros(case.n_dofs)
    op.evaluate_residual_plain(res, np.ascontiguousarray(case.u_star[perm]))
    assert rel_err(res, o.evaluate_residual(case.u_star)[perm]) < 1e-12
    d = np.zeros(case.n_dofs)
    op.compute_inverse_diagonal(d)
    assert rel_err(d, o.inverse_diagonal()[perm]) < 1e-11
    umax = op.get_max_u(np.ascontiguousarray(case.u_star[perm]))
    assert abs(umax - o.get_max_u(case.u_star)) < 1e-13 * umax
    # device memory, caller numbering
    op2 = case.gpu("f64")
    op2.set_vector_layout("device", perm)
    op2.set_linearization_point(case.u_star[perm])
    op2.set_previous_solution([h[perm] for h in case.hist], case.weights)
    y = op2.initialize_dof_vector()
    op2.vmult(y, op2._dev(case.src[perm]))
    torch.cuda.synchronize()
    assert rel_err(y.cpu().numpy(), dst) < 1e-13  # LDS-atomic summation order only


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_get_max_u(prec):
    case = deck_case("input_turek_2D_Re100.json", 2)
    o = case.oracle()
    op = case.gpu(prec)
    for v in (case.u_star, case.src):
        got = op.get_max_u(op._dev(v))
        ref = o.get_max_u(v)
        assert abs(got - ref) < (1e-13 if prec == "f64" else 1e-6) * ref


@pytest.mark.parametrize("layout", ["device", "host"])
def test_vmult_interface_down_up(layout):
    """vmult_interface_down / _up (operator_ns.cc:734-787) on a globally
    refined level, where no dof sits on a refinement edge: down is the vmult
    (the oracle's, identity rows included), up overwrites dst with zeros."""
    import torch
    case = deck_case("input_hoffmann_3D_Re3900.json", 1)
    ref = case.oracle().vmult(case.src)
    op = case.gpu("f64")
    if layout == "host":
        op.set_vector_layout("host", None)
        src, down, up = case.src.copy(), np.full(case.n_dofs, 7.0), np.full(case.n_dofs, 7.0)
        op.vmult_interface_down(down, src)
        op.vmult_interface_up(up, src)
    else:
        src = op._dev(case.src)
        down = op.initialize_dof_vector().fill_(7.0)
        up = op.initialize_dof_vector().fill_(7.0)
        op.vmult_interface_down(down, src)
        op.vmult_interface_up(up, src)
        torch.cuda.synchronize()
        down, up = down.cpu().numpy(), up.cpu().numpy()
    assert rel_err(down, ref) < 1e-12
    assert not np.any(up)


def test_multigrid_and_gmres_host_permuted():
    import torch
    import glsamd
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(2)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                             coarse_n_iterations=10)
    n = meshes[-1].n_dofs
    b = gi.rnd(3, n)
    ref = torch.zeros(n, dtype=torch.float64, device="cuda")
    mg.vcycle(ref, torch.from_numpy(b).cuda())
    torch.cuda.synchronize()
    perm = _perm(n, 9)
    mg.set_vector_layout("host", perm)
    out = np.zeros(n)
    mg.vcycle(out, np.ascontiguousarray(b[perm]))
    assert rel_err(out, ref.cpu().numpy()[perm]) < 1e-6  # FP32 levels, atomic order
    # GMRES with the host / permuted operator and the host / permuted V-cycle
    # layout (the solver stages x and b once; inside everything is device)
    A = glsamd.NavierStokesOperator(meshes[-1], cm[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    xd = A.initialize_dof_vector()
    lin = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-6)
    mg.set_vector_layout("device")
    lin.solve(xd, A._dev(b))
    torch.cuda.synchronize()
    it_dev = lin.last["n_iterations"]
    A.set_vector_layout("host", perm)
    xh = np.zeros(n)
    lin.solve(xh, np.ascontiguousarray(b[perm]))
    assert abs(lin.last["n_iterations"] - it_dev) <= 1
    assert rel_err(xh, xd.cpu().numpy()[perm]) < 1e-5
