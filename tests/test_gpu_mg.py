"""GPU geometric multigrid (csrc/mg.hip through the C-ABI) vs the oracle-based
CPU multigrid (tests/mg_ref.py) on the same level hierarchy and inputs.

Level operators run in FP32 (MGNumber = float, config.h:7); the oracle runs
in FP64, so the tolerances are FP32-level: transfers 1e-6, smoother /
V-cycle 1e-4 relative l2, relaxation factor 1e-3 relative."""
import numpy as np
import pytest

import glsinputs as gi
from helpers import deck, rel_err
from mg_ref import OracleGMG

pytestmark = pytest.mark.gpu


def _hierarchy(name, n_ref):
    d = deck(name)
    meshes = [d.mesh(r) for r in range(n_ref + 1)]
    vel, p, slip = d.boundary_descriptor()
    cmasks = [m.constraint_mask(vel, p, slip) for m in meshes]
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(meshes[-1].n_nodes, meshes[-1].dim, d.u_max)
    hist = gi.history(u, params["order"])
    return meshes, cmasks, params, w, u, hist


def _np(t):
    return t.double().cpu().numpy()


CASES = [("input_turek_2D_Re20_stat.json", 2), ("input_hoffmann_3D_Re3900.json", 1),
         ("input_turek_2D_Re100.json", 2)]


@pytest.mark.parametrize("name,n_ref", CASES)
def test_transfer(name, n_ref):
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy(name, n_ref)
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32")
    ref = OracleGMG(meshes, cmasks, params, u, hist, w)
    for l in range(1, len(meshes)):
        xc = gi.rnd(5 + l, meshes[l - 1].n_dofs)
        xf = gi.rnd(7 + l, meshes[l].n_dofs)
        pf = ops[l].initialize_dof_vector()
        mg.prolongate_add(l, pf, ops[l - 1]._dev(xc))
        rc = ops[l - 1].initialize_dof_vector()
        mg.restrict_add(l, rc, ops[l]._dev(xf))
        ic = ops[l - 1].initialize_dof_vector()
        mg.interpolate(l, ic, ops[l]._dev(xf))
        torch.cuda.synchronize()
        pref = np.zeros(meshes[l].n_dofs)
        ref.prolongate_add(l, pref, xc)
        rref = np.zeros(meshes[l - 1].n_dofs)
        ref.restrict_add(l, rref, xf)
        assert rel_err(_np(pf), pref) < 1e-6
        assert rel_err(_np(rc), rref) < 1e-6
        assert rel_err(_np(ic), ref.interpolate(l, xf)) < 1e-7


@pytest.mark.parametrize("name,n_ref,coarse", [
    ("input_turek_2D_Re20_stat.json", 2, -1),   # dense LU coarse solve ("direct")
    ("input_turek_2D_Re100.json", 2, -1),       # direct, a third of the coarse dofs constrained
    ("input_turek_2D_Re20_stat.json", 2, 0),    # identity coarse solve
    ("input_hoffmann_3D_Re3900.json", 1, 10),   # relaxation sweeps
])
def test_relaxation_and_vcycle(name, n_ref, coarse):
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy(name, n_ref)
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32",
                               coarse_n_iterations=coarse)
    ref = OracleGMG(meshes, cmasks, params, u, hist, w, coarse_iters=coarse)
    # power-iteration relaxation factor (deal.II start vector, FP32 vs FP64);
    # estimated on the levels above the coarsest (multigrid.cc:355-358) and on
    # the coarse level only when the relaxation coarse solve uses it
    for l in range(len(meshes)):
        omega, lam = mg.relaxation(l)
        if l == 0 and coarse <= 0:
            assert lam == 0.0 and omega == 1.0
            continue
        lam_ref = ref.estimate(l)
        assert abs(lam - lam_ref) < 1e-3 * lam_ref
        assert abs(omega - 2.0 / (lam / 20.0 + lam)) < 1e-12 * omega
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
    # one smoother application on the finest level (vmult from zero)
    L = len(meshes) - 1
    b = gi.rnd(11, meshes[L].n_dofs)
    x = ops[L].initialize_dof_vector()
    mg.smooth(L, x, ops[L]._dev(b), True)
    torch.cuda.synchronize()
    xr = ref.smooth(L, None, b, True, 5)
    assert rel_err(_np(x), xr) < 1e-4
    # full V-cycle, FP64 in / out (copy_to_mg / copy_from_mg)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    # FP32 levels vs FP64 oracle; the stationary saddle-point deck amplifies
    # round-off through the coarse LU (entries up to ~1e3 for O(1) input)
    assert rel_err(_np(dst), ref.vcycle(b)) < 5e-4


@pytest.mark.parametrize("name,n_ref,tol", [("input_turek_2D_Re20_stat.json", 2, 2e-3),
                                            ("input_hoffmann_3D_Re3900.json", 1, 1e-6)])
def test_level_diagonals(name, n_ref, tol):
    """Inverse diagonals of the FP32 level operators (set up by build_gmg on
    interpolated linearization points) against the oracle multigrid's FP64
    ones.  The stationary Re20 saddle-point operator has near-cancelling
    diagonal entries (|1/d| up to 1.4e5): FP32 table rounding gives 7.7e-4
    relative l2 on its coarse level with the direct element-diagonal kernel,
    1.1e-3 with unit-vector cell applies (round 1, measured,
    scripts/diag_check.py); the FP64 level operators agree to 1e-11."""
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy(name, n_ref)
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32")
    ref = OracleGMG(meshes, cmasks, params, u, hist, w)
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        assert rel_err(_np(dl), ref.invdiag[l]) < tol


def _gmres(apply_A, apply_P, b, iters):
    """Right-preconditioned GMRES without restart (test harness only; the
    reference's LinearSolverGMRES, solver_l.cc:45-74, is out of scope)."""
    import torch
    beta = b.norm()
    V = [b / beta]
    Z = []
    H = torch.zeros(iters + 1, iters, dtype=torch.float64)
    res = [1.0]
    for j in range(iters):
        z = apply_P(V[j])
        Z.append(z)
        w = apply_A(z)
        for i in range(j + 1):
            H[i, j] = float(torch.dot(w, V[i]))
            w = w - H[i, j] * V[i]
        H[j + 1, j] = float(w.norm())
        V.append(w / H[j + 1, j])
        e1 = torch.zeros(j + 2, dtype=torch.float64)
        e1[0] = float(beta)
        y = torch.linalg.lstsq(H[:j + 2, :j + 1], e1).solution
        res.append(float((H[:j + 2, :j + 1] @ y - e1).norm() / beta))
    return res


def test_vcycle_preconditions_gmres():
    """The V-cycle is a useful preconditioner for the deck's Newton operator:
    right-preconditioned GMRES reduces the residual much faster than
    unpreconditioned GMRES (PreconditionerGMG inside LinearSolverGMRES)."""
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 1)
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32",
                               coarse_n_iterations=10)
    A = glsamd.NavierStokesOperator(meshes[-1], cmasks[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    b = A._dev(gi.rnd(3, meshes[-1].n_dofs))

    def apply_A(x):
        y = torch.empty_like(x)
        A.vmult(y, x)
        return y

    def apply_P(x):
        y = torch.empty_like(x)
        mg.vcycle(y, x)
        return y

    plain = _gmres(apply_A, lambda x: x, b, 20)
    prec = _gmres(apply_A, apply_P, b, 20)
    torch.cuda.synchronize()
    print("gmres plain", plain[-1], "gmg", prec[-1])
    # measured: 6.2e-3 after 20 iterations with a two-level FP32 V-cycle
    assert prec[-1] < 1e-2, prec
    assert prec[-1] < 0.25 * plain[-1], (prec[-1], plain[-1])


@pytest.mark.parametrize("name,n_ref,coarse", [("input_turek_2D_Re20_stat.json", 2, -1),
                                               ("input_sphere_amg.json", 1, 10)])
def test_coarse_gmres_vcycle(name, n_ref, coarse):
    """The AMG decks' "gmg coarse grid iterate" (multigrid.cc:491-530): GMRES
    to 1e-4 on the coarse level inside the V-cycle, preconditioned by the
    substitute for Trilinos AMG: the dense LU on the
    stationary saddle-point deck (Jacobi sweeps diverge there), 10 relaxation
    sweeps on the sphere; against the oracle multigrid's restatement on the
    GPU's own omegas/diagonals."""
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy(name, n_ref)
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32",
                               coarse_n_iterations=coarse, coarse_iterate=True,
                               coarse_reltol=1e-4, coarse_maxiter=500)
    ref = OracleGMG(meshes, cmasks, params, u, hist, w, coarse_iters=coarse,
                    coarse_gmres_reltol=1e-4)
    ref.set_omega([mg.relaxation(l)[0] for l in range(len(meshes))])
    for l in range(len(meshes)):
        dl = ops[l].initialize_dof_vector()
        ops[l].compute_inverse_diagonal(dl)
        ref.invdiag[l] = _np(dl)
    L = len(meshes) - 1
    b = gi.rnd(11, meshes[L].n_dofs)
    src = torch.from_numpy(b).cuda()
    dst = torch.zeros_like(src)
    mg.vcycle(dst, src)
    torch.cuda.synchronize()
    it, conv = mg.coarse_statistics()
    xr = ref.vcycle(b)
    assert conv and it > 0
    assert abs(it - ref.coarse_gmres_iterations) <= 3, (it, ref.coarse_gmres_iterations)
    assert rel_err(_np(dst), xr) < 2e-3


def _re3900_gmg(coarse, prec="f32"):
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
    mg, ops = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision=prec,
                               coarse_n_iterations=coarse)
    A = glsamd.NavierStokesOperator(meshes[-1], cmasks[-1], "f64")
    A.set_parameters(**params)
    A.set_linearization_point(u)
    A.set_previous_solution(hist, w)
    return meshes, mg, A


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_coarse_inverse_trtri_vs_getrs(prec, monkeypatch):
    """The dense coarse solver's inverse (multigrid.cc:448-455 substitute):
    the default Z = U^-1 L^-1 (rocsolver_dtrtri + rocblas_dtrsm, pivots
    applied to the GEMV's input gather) against getrs with the identity
    (the round-3 path), on the headline hierarchy r0..r2: the V-cycles agree
    to the FP64 rounding of two orderings of the same inverse (FP64 levels,
    5e-12)
    and to the FP32 storage of the inverse (FP32 levels); the setup times of
    both are printed."""
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
    b = gi.rnd(31, meshes[-1].n_dofs)
    out = {}
    for mode in ("getrs", "trtri"):
        if mode == "getrs":
            monkeypatch.setenv("GLS_COARSE_REFERENCE", "getrs")
        else:
            monkeypatch.delenv("GLS_COARSE_REFERENCE", raising=False)
        # deterministic mode: repeated cycles bitwise equal, so the bound
        # below is the inverses' own difference, not run-to-run noise
        mg, _ = glsamd.build_gmg(meshes, cmasks, dict(params, deterministic=True), u, hist, w,
                                 precision=prec, coarse_n_iterations=-1)
        src = torch.from_numpy(b).cuda()
        ys = []
        for _ in range(2):
            dst = torch.zeros_like(src)
            mg.vcycle(dst, src)
            torch.cuda.synchronize()
            ys.append(_np(dst))
        out[mode] = (ys, mg.coarse_setup_times())
        del mg
    err = rel_err(out["trtri"][0][0], out["getrs"][0][0])
    d_ee = rel_err(out["trtri"][0][1], out["trtri"][0][0])
    print(f"{prec}: trtri vs getrs V-cycle {err:.2e} (eager vs eager {d_ee:.1e}); setup "
          f"getrs {out['getrs'][1]}, trtri {out['trtri'][1]}")
    # FP64: two orderings of the same inverse of a coarse matrix whose FP64 LU
    # already differs from the oracle's numpy LU by ~4e-12 in the V-cycle
    # (test_vcycle_re3900_f64_levels_tight[-1]); measured 6.2e-13 - 1.15e-12.
    # FP32: the FP32 copies of the two inverses (measured 2.6e-7 - 2.8e-7;
    # round 4 had to allow 20x the cycle's LDS-atomic run-to-run noise)
    assert d_ee == 0.0
    assert err < (5e-12 if prec == "f64" else 1e-6)


@pytest.mark.parametrize("coarse", [10, -1])
def test_vcycle_deferred_reductions(coarse, monkeypatch):
    """The smoother's deferred shared-node reductions (FP32 3D brick levels:
    each apply's boundary rows rebuilt in the next apply's gather from its
    partial slots, k_shared_reduce_cls's arithmetic; one explicit reduction
    per smoothing sequence, the pre-smoothing's rebuilt by the residual
    apply) against a reduction after every apply (GLS_MG_DEFER=0, read once
    per process: the reference cycle runs in a child process) on the headline
    hierarchy r0..r2.  Same tolerance rule as the graph test: the eager
    cycle's own run-to-run difference (LDS-atomic order) times 20, at least
    1e-6; and the GMRES iteration count."""
    import subprocess
    import sys
    import torch
    import glsamd
    meshes, mg, A = _re3900_gmg(coarse)
    b = gi.rnd(41, meshes[-1].n_dofs)

    def cycle():
        x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
        mg.vcycle(x, torch.from_numpy(b).cuda())
        torch.cuda.synchronize()
        return _np(x)

    y1, y2 = cycle(), cycle()
    x = torch.zeros_like(torch.from_numpy(b)).cuda()
    s = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-8, absolute_tolerance=0.0)
    s.solve(x, torch.from_numpy(b).cuda())
    it = s.last["n_iterations"]
    code = f"""
import sys, numpy as np, torch
sys.path[:0] = {sys.path!r}
import glsamd, glsinputs as gi
from test_gpu_mg import _re3900_gmg
meshes, mg, A = _re3900_gmg({coarse})
b = gi.rnd(41, meshes[-1].n_dofs)
x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
mg.vcycle(x, torch.from_numpy(b).cuda())
s = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-8, absolute_tolerance=0.0)
x2 = torch.zeros_like(x)
s.solve(x2, torch.from_numpy(b).cuda())
torch.cuda.synchronize()
np.save(sys.argv[1], x.cpu().numpy())
print(s.last["n_iterations"])
"""
    import os
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "ref.npy")
        env = dict(os.environ, GLS_MG_DEFER="0")
        r = subprocess.run([sys.executable, "-c", code, f], env=env, capture_output=True,
                           text=True, timeout=180, cwd=os.path.dirname(__file__))
        assert r.returncode == 0, r.stderr[-2000:]
        ref = np.load(f)
        it_ref = int(r.stdout.strip().splitlines()[-1])
    d_ee = rel_err(y2, y1)
    d = rel_err(y1, ref)
    print(f"coarse {coarse}: deferred vs per-apply reductions {d:.1e} (eager vs eager {d_ee:.1e}),"
          f" GMRES {it} vs {it_ref} iterations")
    assert d < max(1e-6, 20 * d_ee)
    assert abs(it - it_ref) <= 1


def test_vcycle_resident_sweeps():
    """The resident smoothing sweeps (k_brick_sweeps: a level's smoothing
    sequence in one launch, bricks waiting only for the bricks they share a
    node with) against one launch per step (GLS_MG_DEFER=1, a child process)
    on the headline hierarchy r0..r2 with 10 coarse sweeps: BITWISE equal
    V-cycles in deterministic mode, also while another stream streams a
    large copy through the device (uneven load on the hand-offs), and no
    neighbour wait hit its spin bound; the GMRES iteration count of the
    default mode within 1 of the per-launch one."""
    import os
    import subprocess
    import sys
    import tempfile
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
    pdet = dict(params, deterministic=True)
    mg, ops = glsamd.build_gmg(meshes, cmasks, pdet, u, hist, w, precision="f32",
                               coarse_n_iterations=10)
    b = gi.rnd(41, meshes[-1].n_dofs)
    bd = torch.from_numpy(b).cuda()

    def cycle():
        x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
        mg.vcycle(x, bd)
        torch.cuda.synchronize()
        return _np(x)

    y1 = cycle()
    # the same cycles with a 1 GiB device copy running on another stream
    big = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    big2 = torch.empty_like(big)
    side = torch.cuda.Stream()
    ys = []
    for _ in range(4):
        with torch.cuda.stream(side):
            big2.copy_(big)
        ys.append(cycle())
        torch.cuda.synchronize()
    del big, big2
    for y in ys:
        assert np.array_equal(y, y1)
    stats = [op.sweep_stats() for op in ops]
    print("resident launches / spin-bound waits per level:", stats)
    assert all(s[1] == 0 for s in stats), stats
    # r0 (coarse sweeps) and r1 (pre- and post-smoothing) ran resident
    assert stats[0][0] > 0 and stats[1][0] > 0, stats
    code = f"""
import sys, numpy as np, torch
sys.path[:0] = {sys.path!r}
import glsamd, glsinputs as gi
from test_gpu_mg import _hierarchy, _re3900_gmg
meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
mg, ops = glsamd.build_gmg(meshes, cmasks, dict(params, deterministic=True), u, hist, w,
                           precision="f32", coarse_n_iterations=10)
b = gi.rnd(41, meshes[-1].n_dofs)
x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
mg.vcycle(x, torch.from_numpy(b).cuda())
np.save(sys.argv[1], x.cpu().numpy())
meshes, mg, A = _re3900_gmg(10)
s = glsamd.LinearSolverGMRES(A, mg, relative_tolerance=1e-8, absolute_tolerance=0.0)
x2 = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
s.solve(x2, torch.from_numpy(b).cuda())
torch.cuda.synchronize()
print(s.last["n_iterations"])
"""
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "launches.npy")
        r = subprocess.run([sys.executable, "-c", code, f], env=dict(os.environ, GLS_MG_DEFER="1"),
                           capture_output=True, text=True, timeout=180,
                           cwd=os.path.dirname(__file__))
        assert r.returncode == 0, r.stderr[-2000:]
        y_launch = np.load(f)
        it_launch = int(r.stdout.strip().splitlines()[-1])
    n_diff = int(np.count_nonzero(y_launch != y1))
    meshes2, mg2, A = _re3900_gmg(10)
    x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
    s = glsamd.LinearSolverGMRES(A, mg2, relative_tolerance=1e-8, absolute_tolerance=0.0)
    s.solve(x, bd)
    it = s.last["n_iterations"]
    print(f"resident sweeps vs one launch per step: {n_diff} entries differ (deterministic); "
          f"GMRES {it} vs {it_launch} iterations")
    assert n_diff == 0
    assert abs(it - it_launch) <= 1


def test_resident_sweep_stall_recovers():
    """A resident smoothing sweep whose neighbour wait gives up (forced with a
    spin bound of 0 polls on every level, gls_op_set_sweep_spin_bound)
    poisons its V-cycle with NaN and raises the level's stall flag; the
    multigrid reports it ONCE as an error status of gls_mg_vcycle and then
    runs one launch per smoothing step for good: the next V-cycles equal the
    resident one bitwise (deterministic mode: resident and per-launch steps
    are the same arithmetic).  Then, on a
    fresh multigrid with the default bound, the cycles run while a
    CU-holding GEMM occupies another stream: either the bricks stay
    co-resident (bitwise the quiet cycle) or the stall is reported once and
    the next cycle is again bitwise right."""
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
    pdet = dict(params, deterministic=True)
    b = torch.from_numpy(gi.rnd(43, meshes[-1].n_dofs)).cuda()

    def cycle(m):
        x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
        m.vcycle(x, b)
        torch.cuda.synchronize()
        return _np(x)

    mg, ops = glsamd.build_gmg(meshes, cmasks, pdet, u, hist, w, precision="f32",
                               coarse_n_iterations=10)
    y_ref = cycle(mg)
    assert np.isfinite(y_ref).all()
    for op in ops:
        op.set_sweep_spin_bound(0)
    errors, outs = 0, []
    for _ in range(3):
        try:
            outs.append(cycle(mg))
        except glsamd.GlsError as e:
            assert "resident smoothing sweep timed out" in str(e), e
            errors += 1
            break
    stats = [op.sweep_stats() for op in ops]
    print("forced stall: launches / spin-bound waits per level", stats, "errors", errors)
    if sum(st[1] for st in stats) == 0:
        pytest.skip("no neighbour wait missed its first poll: the stall path did not trigger")
    assert errors == 1
    # the cycles before the stalled one are intact; the stalled one (the last
    # completed, if its flag showed only at the next call) carries NaN
    assert all(np.array_equal(y, y_ref) for y in outs[:-1])
    launches = [op.sweep_stats()[0] for op in ops]
    for _ in range(2):
        assert np.array_equal(cycle(mg), y_ref)
    assert [op.sweep_stats()[0] for op in ops] == launches  # no resident launch since
    # default bound, a GEMM holding CUs on another stream during the cycles
    mg2, ops2 = glsamd.build_gmg(meshes, cmasks, pdet, u, hist, w, precision="f32",
                                 coarse_n_iterations=10)
    a = torch.randn(8192, 8192, device="cuda")
    side = torch.cuda.Stream()
    reported = 0
    for _ in range(4):
        with torch.cuda.stream(side):
            c = a @ a
        try:
            y = cycle(mg2)
            assert np.array_equal(y, y_ref) or not np.isfinite(y).all()
        except glsamd.GlsError as e:
            assert "resident smoothing sweep timed out" in str(e), e
            reported += 1
        torch.cuda.synchronize()
    del c
    print("concurrent GEMM: stalls reported", reported,
          "stats", [op.sweep_stats() for op in ops2])
    assert reported <= 1
    assert np.array_equal(cycle(mg2), y_ref)


def test_vcycle_deterministic_bitwise():
    """GLS_DETERMINISTIC (SURVEY §7.2.2's deterministic mode): the brick
    kernels add a round's cells into the LDS lattice in cell order instead of
    by LDS atomics, the diagonal and the restriction assemble cell colour by
    colour instead of by global atomics.  On the headline hierarchy r0..r2
    (FP32 levels, 10 coarse sweeps): two setups give bitwise the same
    relaxation factors, repeated V-cycles are bitwise equal, the smoother's
    deferred shared-node reductions equal a reduction after every apply
    (GLS_MG_DEFER=0, a child process) BITWISE -- the rebuild reproduces the
    reduce kernel's arithmetic -- and the FP64 vmult is bitwise repeatable
    and within 1e-12 of the oracle; the default mode stays within FP32
    round-off of it."""
    import os
    import subprocess
    import sys
    import tempfile
    import torch
    import glsamd
    meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
    pdet = dict(params, deterministic=True)
    mg, ops = glsamd.build_gmg(meshes, cmasks, pdet, u, hist, w, precision="f32",
                               coarse_n_iterations=10)
    om1 = [mg.relaxation(l) for l in range(len(meshes))]
    mg.setup()
    om2 = [mg.relaxation(l) for l in range(len(meshes))]
    assert om1 == om2, (om1, om2)
    b = gi.rnd(41, meshes[-1].n_dofs)

    def cycle(m):
        x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
        m.vcycle(x, torch.from_numpy(b).cuda())
        torch.cuda.synchronize()
        return _np(x)

    y1, y2, y3 = cycle(mg), cycle(mg), cycle(mg)
    assert np.array_equal(y1, y2) and np.array_equal(y1, y3)
    code = f"""
import sys, numpy as np, torch
sys.path[:0] = {sys.path!r}
import glsamd, glsinputs as gi
from test_gpu_mg import _hierarchy
meshes, cmasks, params, w, u, hist = _hierarchy("input_hoffmann_3D_Re3900.json", 2)
mg, ops = glsamd.build_gmg(meshes, cmasks, dict(params, deterministic=True), u, hist, w,
                           precision="f32", coarse_n_iterations=10)
b = gi.rnd(41, meshes[-1].n_dofs)
x = torch.zeros(meshes[-1].n_dofs, dtype=torch.float64, device="cuda")
mg.vcycle(x, torch.from_numpy(b).cuda())
torch.cuda.synchronize()
np.save(sys.argv[1], x.cpu().numpy())
"""
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "eager.npy")
        r = subprocess.run([sys.executable, "-c", code, f], env=dict(os.environ, GLS_MG_DEFER="0"),
                           capture_output=True, text=True, timeout=180,
                           cwd=os.path.dirname(__file__))
        assert r.returncode == 0, r.stderr[-2000:]
        y_eager = np.load(f)
    n_diff = int(np.count_nonzero(y_eager != y1))
    print(f"deterministic: deferred vs per-apply reductions differ in {n_diff} entries")
    assert n_diff == 0
    # the default (atomic) mode: within FP32 round-off of the deterministic cycle
    mgd, _ = glsamd.build_gmg(meshes, cmasks, params, u, hist, w, precision="f32",
                              coarse_n_iterations=10)
    d = rel_err(cycle(mgd), y1)
    print(f"default vs deterministic V-cycle {d:.1e}")
    assert d < 1e-5
    # FP64 vmult: bitwise repeatable, oracle parity
    from helpers import Case
    c = Case(meshes[-1], cmasks[-1], params, w, 1.0)
    op = glsamd.NavierStokesOperator(meshes[-1], cmasks[-1], "f64")
    op.set_parameters(**dict(params, deterministic=True))
    op.set_linearization_point(u)
    op.set_previous_solution(hist, w)
    src = op._dev(c.src)
    outs = []
    for _ in range(3):
        dst = op.initialize_dof_vector()
        op.vmult(dst, src)
        torch.cuda.synchronize()
        outs.append(_np(dst))
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    o = c.oracle()
    o.set_linearization_point(u)
    o.set_previous_solution(hist, w)
    assert rel_err(outs[0], o.vmult(c.src)) < 1e-12
