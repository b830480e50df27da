"""GPU parity at every BASELINE.json config's CONFIGURED size (the deck's own
"n global refinements", shift, boundary conditions and time integrator), HIP
path through the C-ABI vs the CPU oracle on the same mesh and §8d synthetic
inputs.  The headline Re3900 r2 vmult is covered by test_gpu_parity.py; this
file adds the larger decks and the headline's full 3-level V-cycle.

Tolerances (relative l2): FP64 1e-12, FP32 2e-5 (operators); the FP32
V-cycle against the FP64 oracle multigrid 5e-4 (test_gpu_mg.py).

Named test_a_* so that these run first under `pytest -x`."""
import numpy as np
import pytest

import glsinputs as gi
from helpers import deck, deck_case, rel_err
from mg_ref import OracleGMG

pytestmark = pytest.mark.gpu
TOL = {"f64": 1e-12, "f32": 2e-5}


def _np(t):
    return t.double().cpu().numpy()


def _vmult(case, prec):
    import torch
    op = case.gpu(prec)
    dst = op.initialize_dof_vector()
    op.vmult(dst, op._dev(case.src))
    torch.cuda.synchronize()
    out = _np(dst)
    del op, dst
    torch.cuda.empty_cache()
    return out


@pytest.fixture(scope="module")
def turek3d_r3():
    # input_turek_3D_Re100.json as configured: r3 (204,800 cells, 6,789,120
    # DoFs), cylinder shift 0.005, no-slip walls, BDF2
    d = deck("input_turek_3D_Re100.json")
    assert d.n_refinements == 3
    case = deck_case("input_turek_3D_Re100.json")
    assert case.n_dofs == 6789120
    o = case.oracle()
    return case, o.vmult(case.src), o.evaluate_residual(case.u_star)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_turek3d_r3_vmult(turek3d_r3, prec):
    case, ref, _ = turek3d_r3
    assert rel_err(_vmult(case, prec), ref) < TOL[prec]


def test_turek3d_r3_residual(turek3d_r3):
    import torch
    case, _, ref = turek3d_r3
    op = case.gpu("f64")
    res = op.initialize_dof_vector()
    op.evaluate_residual_plain(res, op._dev(case.u_star))
    torch.cuda.synchronize()
    assert rel_err(_np(res), ref) < TOL["f64"]


@pytest.fixture(scope="module")
def sphere_r3():
    # input_sphere_amg.json as configured: mesh/sphere.msh r3 (524,288 cells,
    # 17,073,608 DoFs), every cell general geometry
    d = deck("input_sphere_amg.json")
    assert d.n_refinements == 3
    case = deck_case("input_sphere_amg.json")
    assert case.n_dofs == 17073608
    return case, case.oracle().vmult(case.src)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_sphere_r3_vmult(sphere_r3, prec):
    # FP32: the sphere's multigrid levels run the FP32 operator
    case, ref = sphere_r3
    err = rel_err(_vmult(case, prec), ref)
    print(f"sphere r3 {prec} vmult rel err {err:.2e}")
    assert err < TOL[prec]


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_turek2d_re100_r5_vmult(prec):
    # input_turek_2D_Re100.json as configured: Q1, r5 (90,112 cells)
    d = deck("input_turek_2D_Re100.json")
    assert d.n_refinements == 5
    case = deck_case("input_turek_2D_Re100.json")
    ref = case.oracle().vmult(case.src)
    assert rel_err(_vmult(case, prec), ref) < TOL[prec]


def test_vcycle_re3900_r0_r2():
    """The headline hierarchy (Re3900 r0 -> r1 -> r2, FP32 levels): relaxation
    factors, one pre-smoothing and one full V-cycle against the oracle
    multigrid.  Coarse solve: 10 relaxation sweeps — the substitute for the
    deck's Trilinos direct solver, identical on both sides."""
    import torch
    import glsamd
    d = deck("input_hoffmann_3D_Re3900.json")
    meshes = [d.mesh(r) for r in range(d.n_refinements + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=10)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=10)
    for l in range(len(meshes)):
        omega, lam = mg.relaxation(l)
        lam_ref = ref.estimate(l)
        assert abs(lam - lam_ref) < 1e-3 * lam_ref, (l, lam, lam_ref)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    # the relaxation / V-cycle algorithm is compared on the GPU's own FP32
    # level diagonals (MGNumber = float): near-cancelling diagonal entries of
    # the saddle-point operator amplify FP32 table rounding in D^{-1}; the
    # diagonals themselves are checked against the oracle in
    # test_gpu_parity.py::test_inverse_diagonal and test_level_diagonals
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        ref.invdiag[l] = _np(dl)
    L = len(meshes) - 1
    b = gi.rnd(11, meshes[L].n_dofs)
    x = ops[L].initialize_dof_vector()
    mg.smooth(L, x, ops[L]._dev(b), True)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    assert rel_err(_np(x), ref.smooth(L, None, b, True, 5)) < 1e-4
    assert rel_err(_np(dst), ref.vcycle(b)) < 5e-4


def _re3900(n_ref=2, name="input_hoffmann_3D_Re3900.json"):
    d = deck(name)
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    return meshes, cm, params, w, u, hist


def test_level_diagonals_re3900_r2():
    """The FP32 level inverse diagonals of the headline hierarchy r0..r2 (the
    r2 level included) against the oracle multigrid's FP64 ones
    (compute_inverse_diagonal, operator_ns.cc:195-225, on the linearization
    point interpolated level by level, main.cc:772-803)."""
    import glsamd
    meshes, cm, params, w, u, hist = _re3900(2)
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32")
    ref = OracleGMG(meshes, cm, params, u, hist, w)
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        err = rel_err(_np(dl), ref.invdiag[l])
        print(f"Re3900 level r{l} FP32 inverse diagonal rel err {err:.2e}")
        assert err < 1e-6, (l, err)


def test_vcycle_re3900_direct_coarse():
    """The deck's own V-cycle ("gmg coarse grid solver": "direct",
    multigrid.cc:448-455, 465-481) on the headline hierarchy r0..r2, FP32
    levels, FP64 in / out: the GPU's dense coarse solve (free-dof block
    assembled from element matrices, LU-inverted, FP32-stored inverse) and
    the GPU's own FP32 inverse diagonals against the oracle multigrid with
    ITS FP64 diagonals and an FP64 LU of the oracle's coarse matrix.  The
    relaxation factors are the GPU's (checked against the oracle's power
    iteration to 1e-3 in test_vcycle_re3900_r0_r2)."""
    import torch
    import glsamd
    meshes, cm, params, w, u, hist = _re3900(2)
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=-1)
    print("coarse setup", mg.coarse_setup_times())
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=-1)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    err = rel_err(_np(dst), ref.vcycle(b))
    print(f"Re3900 r0..r2 direct-coarse V-cycle rel err {err:.2e}")
    assert err < 5e-4


@pytest.mark.parametrize("coarse", [10, -1])
def test_vcycle_re3900_f64_levels_tight(coarse):
    """The multigrid algorithm itself at a tight tolerance: the headline
    hierarchy r0..r2 with FP64 levels (no FP32 rounding anywhere) against the
    oracle multigrid with ITS OWN FP64 inverse diagonals and coarse solve (10
    relaxation sweeps, or the deck's direct solve: the oracle's FP64 LU
    against the GPU's free-dof inverse).  Only the relaxation factors are
    shared (the GPU's power iteration, checked to 1e-3 against the oracle's
    in test_vcycle_re3900_r0_r2).  The FP32-level tests above compare FP32
    arithmetic against FP64 and need 5e-4; this one bounds the algorithmic
    difference at 1e-9."""
    import torch
    import glsamd
    meshes, cm, params, w, u, hist = _re3900(2)
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f64",
                               coarse_n_iterations=coarse)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=coarse)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    err = rel_err(_np(dst), ref.vcycle(b))
    print(f"Re3900 r0..r2 FP64-level V-cycle (coarse {coarse}) rel err {err:.2e}")
    assert err < 1e-9


def test_vcycle_turek3d_direct_coarse():
    """Config 3's own multigrid (input_turek_3D_Re100.json: GMG over r0..r3,
    "gmg coarse grid solver": "direct", cylinder shift 0.005, no-slip walls,
    main.cc:396-568, multigrid.cc:448-455) at the largest hierarchy the
    oracle multigrid sets up in seconds, r0..r2: FP32 levels with the GPU's
    dense coarse solve against the oracle's FP64 diagonals and FP64 LU, and
    the GPU's relaxation factors against the oracle's power iteration."""
    import torch
    import glsamd
    meshes, cm, params, w, u, hist = _re3900(2, "input_turek_3D_Re100.json")
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=-1)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=-1)
    for l in range(1, len(meshes)):  # (the direct-solved coarsest level is not smoothed)
        lg, lr = mg.relaxation(l)[1], ref.estimate(l)
        assert abs(lg - lr) <= 1e-3 * lr, (l, lg, lr)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    b = gi.rnd(13, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    err = rel_err(_np(dst), ref.vcycle(b))
    print(f"Turek-3D r0..r2 direct-coarse V-cycle rel err {err:.2e}")
    assert err < 5e-4


def test_vcycle_turek3d_f64_levels_tight():
    """Config 3's V-cycle with FP64 levels and the deck's direct coarse
    solve against the oracle multigrid (its own FP64 diagonals and LU; the
    relaxation factors shared): the algorithmic difference at 1e-9."""
    import torch
    import glsamd
    meshes, cm, params, w, u, hist = _re3900(2, "input_turek_3D_Re100.json")
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f64",
                               coarse_n_iterations=-1)
    ref = OracleGMG(meshes, cm, params, u, hist, w, coarse_iters=-1)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    b = gi.rnd(13, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    err = rel_err(_np(dst), ref.vcycle(b))
    print(f"Turek-3D r0..r2 FP64-level V-cycle rel err {err:.2e}")
    assert err < 1e-9


def test_coarse_assembly_element_matrices():
    """The dense coarse solver's free-dof block assembled from the level's
    element matrices (one launch + one scatter per cell colour) against the
    column-by-column assembly from unit-vector vmults
    (GLS_COARSE_REFERENCE=columns), FP64 levels r0..r1: the V-cycles agree."""
    import os
    import torch
    import glsamd
    meshes, cm, params, w, u, hist = _re3900(1)
    b = torch.from_numpy(gi.rnd(11, meshes[-1].n_dofs)).cuda()
    out = {}
    for mode in ("columns", "elements", "getri", "nocond"):
        ref = {"columns": "columns,getri", "getri": "getri", "nocond": "nocond"}.get(mode)
        if ref:
            os.environ["GLS_COARSE_REFERENCE"] = ref
        try:
            mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f64",
                                       coarse_n_iterations=-1)
        finally:
            os.environ.pop("GLS_COARSE_REFERENCE", None)
        print(mode, mg.coarse_setup_times())
        x = torch.zeros_like(b)
        mg.vcycle(x, b)
        torch.cuda.synchronize()
        out[mode] = _np(x)
        del mg, ops
    # the round-2 setup (columns + getri) against the default (element
    # matrices + getrs on the identity): both FP64, the difference is the
    # coarse system's conditioning times the different summation / solve order
    err = rel_err(out["elements"], out["columns"])
    err_inv = rel_err(out["elements"], out["getri"])
    err_cond = rel_err(out["elements"], out["nocond"])
    print(f"element vs column coarse assembly: V-cycle rel diff {err:.2e}; "
          f"U^-1 L^-1 vs getri inverse {err_inv:.2e}; condensed vs uncondensed {err_cond:.2e}")
    assert err < 1e-10 and err_inv < 1e-10 and err_cond < 1e-10


# the oracle multigrid's setup at r3 (inverse diagonals by 108 unit-vector
# cell applies per cell on 524,288 cells, four levels of tables) takes minutes
# on the box's 16 threads: the sphere hierarchy is compared at r2 (65,536 fine
# cells, 2.2 M DoFs); its r3 fine operator is checked by test_sphere_r3_vmult
N_REF_SPHERE_MG = 2


def test_vcycle_sphere_iso_q1():
    """The sphere deck's multigrid: FE_Q_iso_Q1 coarse level
    (main.cc:436-446) under r1..r2, FP32 levels,
    coarse GMRES to 1e-4 ("gmg coarse grid iterate", multigrid.cc:491-530)
    preconditioned by 10 relaxation sweeps (the AMG substitute, DESIGN.md
    A16), against the oracle multigrid with its own FP64 diagonals."""
    import torch
    import glsamd
    import glsmesh as gm
    d = deck("input_sphere_amg.json")
    meshes = [d.mesh(r) for r in range(N_REF_SPHERE_MG + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    mg, ops = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f32",
                               coarse_n_iterations=10, coarse_iso_q1=True,
                               coarse_iterate=True, coarse_reltol=1e-4, coarse_maxiter=2000)
    ref = OracleGMG([gm.IsoQ1Mesh(meshes[0])] + meshes[1:], cm, params, u, hist, w,
                    coarse_iters=10, coarse_gmres_reltol=1e-4)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        print(f"sphere level {l} FP32 inverse diagonal rel err "
              f"{rel_err(_np(dl), ref.invdiag[l]):.2e}")
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    it, conv = mg.coarse_statistics()
    xr = ref.vcycle(b)
    err = rel_err(_np(dst), xr)
    print(f"sphere r{N_REF_SPHERE_MG} iso-Q1 V-cycle rel err {err:.2e}, coarse GMRES {it} vs "
          f"{ref.coarse_gmres_iterations}")
    assert conv and abs(it - ref.coarse_gmres_iterations) <= 3
    assert err < 2e-3


def test_vcycle_sphere_iso_q1_f64_tight():
    """The sphere multigrid algorithm at FP64 levels with a tight coarse
    tolerance (coarse GMRES to 1e-10 on both sides): the GPU V-cycle against
    the oracle multigrid beyond FP32 round-off, so that the 2e-3 of the FP32
    test above bounds only the FP32-vs-FP64 difference."""
    import torch
    import glsamd
    import glsmesh as gm
    d = deck("input_sphere_amg.json")
    meshes = [d.mesh(r) for r in range(N_REF_SPHERE_MG + 1)]
    vel, p, slip = d.boundary_descriptor()
    cm = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, 3, d.u_max)
    hist = gi.history(u, params["order"])
    mg, _ = glsamd.build_gmg(meshes, cm, params, u, hist, w, precision="f64",
                             coarse_n_iterations=10, coarse_iso_q1=True,
                             coarse_iterate=True, coarse_reltol=1e-10, coarse_maxiter=5000)
    ref = OracleGMG([gm.IsoQ1Mesh(meshes[0])] + meshes[1:], cm, params, u, hist, w,
                    coarse_iters=10, coarse_gmres_reltol=1e-10)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    b = gi.rnd(11, meshes[-1].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    it, conv = mg.coarse_statistics()
    xr = ref.vcycle(b)
    err = rel_err(_np(dst), xr)
    print(f"sphere r{N_REF_SPHERE_MG} iso-Q1 FP64-level V-cycle (coarse 1e-10) rel err {err:.2e}, "
          f"coarse GMRES {it} vs {ref.coarse_gmres_iterations}")
    # measured 1.5e-15, 134 vs 134 coarse iterations
    assert conv and abs(it - ref.coarse_gmres_iterations) <= 1
    assert err < 1e-10
