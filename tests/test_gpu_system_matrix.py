"""OperatorBase::get_system_matrix (operator_ns.cc:1407-1430): element
matrices from the device DIAG kernel (one unit-vector cell apply per cell and
local dof, gls_op_element_matrices) against the oracle's orc_cell_matrix, and
the assembled CSR (gls_op_system_matrix) against vmult: A x == vmult(x) on the
same seeded input, constrained rows the identity.

Tolerances: FP64 relative l2 1e-12 (element matrices are per-cell, no
atomics; the CSR sum order differs from vmult's), FP32 2e-5."""
import numpy as np
import pytest

from helpers import deck_case, rel_err

pytestmark = pytest.mark.gpu
TOL = {"f64": 1e-12, "f32": 2e-5}


@pytest.mark.parametrize("name,n_ref", [("input_turek_2D_Re20_stat.json", 0),
                                        ("input_hoffmann_3D_Re3900.json", 0)])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_element_matrices(name, n_ref, prec):
    case = deck_case(name, n_ref)
    o = case.oracle()
    op = case.gpu(prec)
    E = op.element_matrices()
    cells = np.unique(np.linspace(0, op.n_cells - 1, 12).astype(int))
    ref = np.stack([o.cell_matrix(int(c)) for c in cells])
    assert E.shape[0] == op.n_cells
    assert rel_err(E[cells], ref) < TOL[prec]


@pytest.mark.parametrize("name,n_ref", [("input_turek_2D_Re20_stat.json", 1),
                                        ("input_hoffmann_3D_Re3900.json", 0)])
@pytest.mark.parametrize("variant", ["newton", "picard"])
def test_system_matrix_vmult(name, n_ref, variant):
    import torch
    over = {} if variant == "newton" else dict(nonlinear_solver="Picard")
    case = deck_case(name, n_ref, **over)
    o = case.oracle()
    op = case.gpu("f64")
    A = op.system_matrix()
    assert A.shape == (op.n_dofs, op.n_dofs)
    assert np.all(np.diff(A.indptr) > 0)
    # columns sorted per row (deal.II SparsityPattern order)
    for r in range(0, op.n_dofs, max(1, op.n_dofs // 50)):
        c = A.indices[A.indptr[r]:A.indptr[r + 1]]
        assert np.all(np.diff(c) > 0)
    ref = o.vmult(case.src)
    assert rel_err(A @ case.src, ref) < TOL["f64"]
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    torch.cuda.synchronize()
    assert rel_err(A @ case.src, dst.double().cpu().numpy()) < TOL["f64"]
    # the diagonal is compute_diagonal's (before inversion)
    assert rel_err(A.diagonal(), o.diagonal()) < TOL["f64"]


def test_system_matrix_shuffled_cells():
    """Brick discovery permutes the cells internally; the matrices must come
    back in the caller's cell order."""
    from shuffle import ShuffledMesh
    from test_brick_discovery import _case
    from helpers import deck
    name = "input_hoffmann_3D_Re3900.json"
    case = _case(ShuffledMesh(deck(name).mesh(1), seed=11), name)
    o = case.oracle()
    op = case.gpu("f64")
    assert op.brick_shape != (0, 0, 0)
    A = op.system_matrix()
    assert rel_err(A @ case.src, o.vmult(case.src)) < TOL["f64"]
    E = op.element_matrices()
    for c in (0, op.n_cells // 2, op.n_cells - 1):
        assert rel_err(E[c], o.cell_matrix(c)) < TOL["f64"]


@pytest.mark.parametrize("name,n_ref", [("input_turek_2D_Re100.json", 1),
                                        ("input_turek_2D_Re20_stat.json", 1)])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_direct_coarse_solve(name, n_ref, prec):
    """The decks' direct coarse solver (multigrid.cc:448-455) as a one-level
    multigrid (gls_mg, coarse_n_iterations = -1: the free-dof block of the
    level operator LU-factorised and inverted once, one GEMV per solve;
    constrained dofs x_c = b_c) against a dense solve of the assembled FP64
    system matrix (gls_op_system_matrix, identity rows on constrained dofs).
    FP64: 1e-10 relative l2 (getri's inverse vs LAPACK's solve, scaled by the
    conditioning; measured 1.8e-12 / 3.7e-12); FP32 (the FP32 operator's
    columns, an FP32-stored inverse): 2e-4 (measured 1.5e-5 / 1.7e-5)."""
    import torch
    import glsamd
    case = deck_case(name, n_ref)
    op = case.gpu(prec)
    A = case.gpu("f64").system_matrix().toarray()
    mg = glsamd.Multigrid([op], [], coarse_n_iterations=-1, outer_precision="f64")
    mg.setup()
    b = np.random.default_rng(5).standard_normal(op.n_dofs)
    x = torch.zeros(op.n_dofs, dtype=torch.float64, device="cuda")
    mg.vcycle(x, torch.from_numpy(b).cuda())
    torch.cuda.synchronize()
    ref = np.linalg.solve(A, b)
    err = rel_err(x.cpu().numpy(), ref)
    print(name, prec, "direct coarse solve rel err", err)
    assert err < (1e-10 if prec == "f64" else 2e-4)
